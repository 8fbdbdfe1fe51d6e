cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6.py tests/test_gpu_parity.py tests/test_gpu_hand.py tests/test_gpu_pipeline.py > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for v in cur base cur base; do
  if [ $v = cur ]; then L=pytorch-openpose_amd/lib/libopose.so; else L=alt_lib/$v.so; fi
  OPOSE_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 5 > gpurun_out/b_$v.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/b_$v.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']; print('$v', round(d['value'],1), d['latency_ms_single_frame'], s.get('maxpool'), s['conv3x3'], s['conv7x7'])"
done
