#!/bin/bash
# build an experimental variant library: tools/build_variant.sh <name> <extra hipcc flags...>
set -e
name=$1; shift
out=/root/repo/mc-path-tracer_amd/build_$name
mkdir -p $out
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -I/root/repo/include -I/root/repo/mc-path-tracer_amd/csrc $@"
pids=()
for f in kernels.hip bvh_build.hip env_build.hip runtime.cpp host/scene.cpp host/proxies.cpp host/capi_host.cpp host/image_io.cpp; do
  /opt/rocm/bin/hipcc $F -x hip -c /root/repo/mc-path-tracer_amd/csrc/$f -o $out/$(basename $f).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed (job $p)" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /root/repo/mc-path-tracer_amd/libmcpt_$name.so $out/*.o
rm -rf $out
