#!/bin/bash
# Round-end measurement pass on the gpurun box: every config's bench line,
# rocprofv3 kernel traces, PMC passes (the inputs of profiles/pmc.json), the
# native gather's per-frame times, the GPU suite and smoke.  Each GPU step
# has its own limit; a timeout, abort or crash ends the pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_session.sh
STEPS="${PASS_STEPS:-bench_all profs pmcs gather}"
for s in $STEPS; do
  case $s in
    bench_all) STEPS=bench_all bash $S || exit $? ;;
    profs) for c in ${PROF_CONFIGS:-c2 c3 c5 c4s9 c3r}; do CONFIG=$c STEPS=prof bash $S || exit $?
             # the line's roofline.kernel must be rocprof's dominant kernel
             python tools/check_kernel_label.py gpurun_out/prof_$c | tee -a gpurun_out/kernel_labels.log || exit 1
           done ;;
    pmcs) for c in ${PMC_CONFIGS:-c2 c3 c4 c4s7 c4s9 c5}; do CONFIG=$c STEPS=pmc bash $S || exit $?; done
          CONFIG=c3r STEPS=pmcx bash $S || exit $? ;;
    gather) timeout -k 10 120 ray-tracing-gpu_amd/lib/rt_render tests/golden/scenes/scene2.dat -x 1920 -y 1080 -d 3 \
              -g 1 --gather rccl -n 50 -o /tmp/g.ppm > gpurun_out/gather_c2_n50.log 2>&1 || exit $? ;;
    tests) STEPS="tests smoke" bash $S || exit $? ;;
  esac
done
exit 0
