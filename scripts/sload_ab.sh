# conv1_1 weights: LDS broadcasts (default build) vs scalar loads (alt_lib/sload.so)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
OPOSE_LIB=alt_lib/sload.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6.py tests/test_gpu_records.py > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for L in pytorch-openpose_amd/lib/libopose.so alt_lib/sload.so pytorch-openpose_amd/lib/libopose.so alt_lib/sload.so; do
  OPOSE_LIB=$L BENCH_PIPELINE=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 --detail > gpurun_out/sl.log 2>&1 || exit 1
  echo "$L $(grep conv1_1 gpurun_out/sl.log | awk '{print $2, $3}') $(python -c "
import json; d=json.loads([l for l in open('gpurun_out/sl.log') if l.startswith('{')][-1]); print(round(d['value'],1), round(d['ms_per_step'],3))")"
done
