#!/bin/bash
# A/B of the big-list kernel's per-wave camera path (camera_buffer=0) and
# default path for the variant libraries VARS in lib/var (first = reference),
# then the GPU suite against TESTLIB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/ray-tracing-gpu_amd/lib/var
for c in ${CONFIGS:-c3 c5}; do
  libs=""; for v in $VARS; do libs="$libs $V/librt_amd_$v.so@camera_buffer=0"; done
  for v in $VARS; do libs="$libs $V/librt_amd_$v.so"; done
  timeout -k 10 400 python tools/ab_variants.py --config $c $libs > gpurun_out/ab_camw_$c.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_camw_$c.log
done
if [ -n "$TESTLIB" ]; then
  RT_AMD_LIB=$V/librt_amd_$TESTLIB.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TESTLIB.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_$TESTLIB.log; exit $rc
fi
