cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/ray-tracing-gpu_amd/lib/var
for c in c3 c5; do
  timeout -k 10 400 python tools/ab_variants.py --config $c $V/librt_amd_base.so@camera_buffer=0 $V/librt_amd_camw.so@camera_buffer=0 $V/librt_amd_base.so $V/librt_amd_camw.so > gpurun_out/ab_camw_$c.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_camw_$c.log
done
for v in base camw; do
  RT_AMD_LIB=$V/librt_amd_$v.so timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_camw_${v}_c3.log 2>&1 || exit 1
  python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/bench_camw_${v}_c3.log') if l.startswith('{')][0]; print('$v', d['kernel_ms'], d['moving_camera_async_ms'], d['frame_costs']['progressive']['stream_fps'])"
done
RT_AMD_LIB=$V/librt_amd_camw.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_camw.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_camw.log; exit $rc
