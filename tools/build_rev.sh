#!/bin/bash
# build the product library of a git revision into mc-path-tracer_amd/libmcpt_<name>.so (A/B baselines):
#   tools/build_rev.sh <name> <rev> [extra hipcc flags...]
set -e
name=$1; rev=$2; shift 2
wt=/tmp/mcpt_wt_$name
rm -rf $wt && git -C /root/repo worktree add -f --detach $wt $rev > /dev/null
out=$wt/build
mkdir -p $out
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -I$wt/include -I$wt/mc-path-tracer_amd/csrc $@"
pids=()
for f in kernels.hip bvh_build.hip env_build.hip runtime.cpp host/scene.cpp host/proxies.cpp host/capi_host.cpp host/image_io.cpp; do
  /opt/rocm/bin/hipcc $F -x hip -c $wt/mc-path-tracer_amd/csrc/$f -o $out/$(basename $f).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /root/repo/mc-path-tracer_amd/libmcpt_$name.so $out/*.o
git -C /root/repo worktree remove --force $wt
