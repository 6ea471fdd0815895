#!/bin/bash
# A/B session on the gpurun box: ab_variants over CONFIGS for the variant
# libraries in lib/var (VARS, in order; the first is the reference), then the
# GPU suite against TESTLIB (a variant name, optional), then read-request /
# write PMC passes of bench.py for PMCCONF x PMCLIBS.  Every GPU step has its
# own time limit and a failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/ray-tracing-gpu_amd/lib/var
libs=""; for v in ${VARS:-base}; do libs="$libs $V/librt_amd_$v.so"; done
for c in ${CONFIGS:-c2}; do
  timeout -k 10 300 python tools/ab_variants.py --config $c $libs > gpurun_out/ab_$c.log 2>&1 || { tail -5 gpurun_out/ab_$c.log; exit 1; }
  tail -1 gpurun_out/ab_$c.log
done
if [ -n "$TESTLIB" ]; then
  RT_AMD_LIB=$V/librt_amd_$TESTLIB.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TESTLIB.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_$TESTLIB.log; [ $rc -eq 0 ] || exit $rc
fi
for c in $PMCCONF; do
  for v in $PMCLIBS; do
    B="python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-boundary --config $c"
    D=gpurun_out/pmc_${c}_$v
    RT_AMD_LIB=$V/librt_amd_$v.so timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $D -o rdreq -- $B > $D.log 2>&1 || exit 1
    RT_AMD_LIB=$V/librt_amd_$v.so timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D -o write -- $B >> $D.log 2>&1 || exit 1
    python tools/pmc_summary.py $D > $D/summary.json && grep -E '"(hbm|read)_bytes_per_launch"' $D/summary.json | tr -d '\n'; echo " $c $v"
  done
done
exit 0
