#!/bin/bash
# Build librt_amd variants for tools/ab_variants.py: name=DEFINES pairs, e.g.
#   tools/build_variants.sh base="-DRT_LB_WAVE_MULTI=0" wm="-DRT_LB_WAVE_MULTI=1"
# -> ray-tracing-gpu_amd/lib/var/librt_amd_<name>.so (parallel builds)
set -e
cd "$(dirname "$0")/../ray-tracing-gpu_amd"
mkdir -p lib/var
rm -f lib/var/*.so
FLAGS="-std=c++17 -O3 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -w"
pids=()
for spec in "$@"; do
  name="${spec%%=*}"; defs="${spec#*=}"
  /opt/rocm/bin/hipcc $FLAGS $defs --offload-arch=gfx950 -shared -o lib/var/librt_amd_$name.so \
      csrc/rt_kernels.hip csrc/rt_scene.cpp csrc/rt_cpu.cpp -Wl,-rpath,/opt/rocm/lib &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la lib/var
