# Measurement pass on the GPU box: PART=1 bench lines of every config (with
# the CPU baselines), PART=2 rocprofv3 kernel traces + PMC for C2/C3/C5 and C4 scene7/scene9 (CONFIGS=...).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
if [ "${PART:-1}" = 1 ]; then
  STEPS="bench_all" bash tools/gpu_session.sh || exit $?
  STEPS="bench" bash tools/gpu_session.sh || exit $?
else
  for c in ${CONFIGS:-c2 c3 c5 c4s7 c4s9}; do CONFIG=$c STEPS="prof pmc" bash tools/gpu_session.sh || exit $?; done
fi
