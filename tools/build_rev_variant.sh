#!/bin/bash
# Build the library of a git revision as an A/B variant: tools/build_rev_variant.sh <name> [rev]
# -> mc-path-tracer_amd/libmcpt_<name>.so (rev defaults to HEAD; the working tree is untouched).
set -e
name=$1
rev=${2:-HEAD}
wt=$(mktemp -d /tmp/mcpt_rev.XXXXXX)
git -C /root/repo worktree add -f "$wt" "$rev" > /dev/null
trap 'git -C /root/repo worktree remove --force "$wt" 2>/dev/null || rm -rf "$wt"' EXIT
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -I$wt/include -I$wt/mc-path-tracer_amd/csrc"
mkdir -p "$wt/b"
pids=()
for f in kernels.hip bvh_build.hip env_build.hip runtime.cpp host/scene.cpp host/proxies.cpp host/capi_host.cpp host/image_io.cpp; do
  /opt/rocm/bin/hipcc $F -x hip -c "$wt/mc-path-tracer_amd/csrc/$f" -o "$wt/b/$(basename $f).o" &
  pids+=($!)
done
# a bare `wait` returns 0 even when a compile failed: wait on each job and stop at a failure
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed (job $p)" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /root/repo/mc-path-tracer_amd/libmcpt_$name.so "$wt"/b/*.o
