# FETCH_SIZE (and kernel time) of tools/build_variants.sh builds: bash tools/pmc_variants.sh CONFIG VARIANTS...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
cfg=$1; shift
for v in "$@"; do
  L=$PWD/ray-tracing-gpu_amd/lib/var/librt_amd_$v.so
  RT_AMD_LIB=$L timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcvar_$cfg/$v -o fetch -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-boundary --config $cfg > gpurun_out/pmcvar_${cfg}_$v.log 2>&1 || exit $?
  python tools/pmc_summary.py gpurun_out/pmcvar_$cfg/$v > gpurun_out/pmcvar_$cfg/$v.json || exit $?
  echo "$v $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/pmcvar_${cfg}_$v.log) $(grep FETCH gpurun_out/pmcvar_$cfg/$v.json)"
done
