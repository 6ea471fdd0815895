# SQ counters of the bounce kernel with and without lane refill
# (RT_OPT_BOUNCE_REFILL): bash tools/refill_pmc.sh c4s7 c4s9
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
for cfg in "$@"; do
  for r in 0 1; do
    D=gpurun_out/refill_pmc_${cfg}_r$r
    B="python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-boundary --config $cfg --option bounce_refill=$r"
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $D -o sq -- $B > $D.sq.log 2>&1 || exit $?
    timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH --output-format csv -d $D -o sq2 -- $B > $D.sq2.log 2>&1 || exit $?
    timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D -o fetch -- $B > $D.fetch.log 2>&1 || exit $?
    timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D -o write -- $B > $D.write.log 2>&1 || exit $?
    K=rt_trace_kernel; [ $r = 1 ] && K=rt_refill_kernel
    python tools/pmc_summary.py $D $K > $D/summary.json || exit $?
    echo "$cfg refill=$r $(grep -o '"kernel_ms": [0-9.]*' $D.sq.log)"
  done
done
