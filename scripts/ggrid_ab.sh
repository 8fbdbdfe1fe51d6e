# gauss_nms grid cap vs the pipelined bench (the NMS shares the chip with the next step's trunk)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
OPOSE_GAUSS_GRID=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_records.py tests/test_gpu_gauss_screen.py tests/test_gpu_parity.py > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for g in 0 512 256 128 0 256 128 64; do
  OPOSE_GAUSS_GRID=$g timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/gg_$g.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/gg_$g.log') if l.startswith('{')][-1]); print('grid=$g', round(d['value'],1), round(d['ms_per_step'],3), d['stage_ms_per_step']['gauss_nms'])"
done
