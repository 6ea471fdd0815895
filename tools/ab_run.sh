# A/B of tools/build_variants.sh builds on the GPU box: bash tools/ab_run.sh LOG CONFIGS VARIANTS...
set -o pipefail
log=gpurun_out/$1; cfgs=$2; shift 2
V="ray-tracing-gpu_amd/lib/var"
libs=""; for v in "$@"; do libs="$libs $V/librt_amd_$v.so"; done
for c in $cfgs; do
  timeout -k 10 240 python -u tools/ab_variants.py --config $c $libs >> $log 2>&1 || exit $?
done
grep config $log
