#!/bin/bash
# One GPU session on the gpurun box: parity tests, smoke, bench, rocprof.
# Every GPU step has its own time limit; a timeout / crash / abort stops the
# session (no further GPU work), an ordinary test failure does not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${STEPS:-tests smoke bench prof}"
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "!! stopping session after $name (rc=$rc)"; exit $rc
  fi
  return 0
}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread ;;
    tests_k) run pytest_gpu_k 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread -k "$TESTK" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py ;;
    bench_all)
      for c in ${CONFIGS:-c1 c2 c3 c4 c4s7 c4s9 c5 c3r c5r}; do run bench_$c 400 python bench.py --config $c --cpu-seconds 5; done ;;
    bench_big)
      for c in ${CONFIGS:-c3 c5}; do run bench_$c 400 python bench.py --config $c --steps 10 --no-cpu-baseline; done ;;
    bench_one) run bench_${CONFIG:-c2} 400 python bench.py --config ${CONFIG:-c2} --steps 20 --no-cpu-baseline ;;
    listpmc) run list_counters 120 rocprofv3 -L ;;
    pmc)
      B="python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-boundary --config ${CONFIG:-c2}"
      run pmc_fetch_${CONFIG:-c2} 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${CONFIG:-c2} -o fetch -- $B
      run pmc_write_${CONFIG:-c2} 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${CONFIG:-c2} -o write -- $B
      run pmc_rdreq_${CONFIG:-c2} 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/pmc_${CONFIG:-c2} -o rdreq -- $B
      run pmc_sq_${CONFIG:-c2} 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_${CONFIG:-c2} -o sq -- $B
      run pmc_sq2_${CONFIG:-c2} 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc_${CONFIG:-c2} -o sq2 -- $B
      python tools/pmc_summary.py gpurun_out/pmc_${CONFIG:-c2} > gpurun_out/pmc_${CONFIG:-c2}/summary.json
      ;;
    pmcx)  # cache and SQ counters per kernel of a config (every kernel kept: tools/pmc_kernels.py)
      B="python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-boundary --config ${CONFIG:-c2}"
      run pmcx_l2_${CONFIG:-c2} 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d gpurun_out/pmcx_${CONFIG:-c2} -o l2 -- $B
      run pmcx_sq_${CONFIG:-c2} 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU --output-format csv -d gpurun_out/pmcx_${CONFIG:-c2} -o sq -- $B
      run pmcx_wr_${CONFIG:-c2} 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcx_${CONFIG:-c2} -o wr -- $B
      run pmcx_fe_${CONFIG:-c2} 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcx_${CONFIG:-c2} -o fe -- $B
      python tools/pmc_kernels.py gpurun_out/pmcx_${CONFIG:-c2} > gpurun_out/pmcx_${CONFIG:-c2}/kernels.json
      ;;
    valumix)  # dynamic VALU instruction mix of a config's kernels
      B="python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-boundary --config ${CONFIG:-c2}"
      run valumix_${CONFIG:-c2} 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --output-format csv -d gpurun_out/valumix_${CONFIG:-c2} -o mix -- $B
      run valumix2_${CONFIG:-c2} 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_IOPS --output-format csv -d gpurun_out/valumix_${CONFIG:-c2} -o mix2 -- $B
      python tools/pmc_kernels.py gpurun_out/valumix_${CONFIG:-c2} > gpurun_out/valumix_${CONFIG:-c2}/kernels.json
      ;;
    ab) run ab_${CONFIG:-c2} 600 python tools/ab_variants.py --config ${CONFIG:-c2} ray-tracing-gpu_amd/lib/var/*.so ;;
    abenv) run abenv_${CONFIG:-c2} 600 python tools/ab_variants.py --config ${CONFIG:-c2} $AB_ARGS ;;
    pmcvar)
      for L in ray-tracing-gpu_amd/lib/var/*.so; do
        n=$(basename $L .so)
        export RT_AMD_LIB=$PWD/$L
        run pmcvar_$n 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcvar/$n -o sq -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --config ${CONFIG:-c2}
        unset RT_AMD_LIB
      done ;;
    fastmath) run fastmath_check 600 tools/fastmath_check ;;
    camprobe)
      for c in ${CONFIGS:-c2 c3}; do
        run camprobe_${c} 300 python tools/camera_probe.py --config $c
        run camprobe_${c}_nocb 300 python tools/camera_probe.py --config $c --cb 0
      done ;;
    camprof)
      for c in ${CONFIGS:-c2 c3}; do
        P=gpurun_out/camprof_$c
        run camprof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run -- python tools/camera_probe.py --config $c
      done ;;

    prof) P=gpurun_out/prof_${CONFIG:-c2}
          run rocprof_${CONFIG:-c2} 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run -- python bench.py --steps ${PROF_STEPS:-200} --no-cpu-baseline --no-host-boundary --config ${CONFIG:-c2}
          python tools/prof_summary.py $P/run_kernel_trace.csv > $P/summary.json
          grep '^{"metric"' gpurun_out/rocprof_${CONFIG:-c2}.log > $P/bench_under_rocprof.json ;;
  esac
done
exit 0
