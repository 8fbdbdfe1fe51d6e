# Small-problem tile cost weights (default) vs the big-grid weights everywhere
# (OPOSE_X6_SMALL_OVH=0): parity tests, then C2 single-frame, C3 Hand(), C5 single-frame
# latencies and the bench line for each.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_hand.py tests/test_gpu_scale_shard.py tests/test_gpu_records.py > gpurun_out/pt_t.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pt_t.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_t.log | head; exit $rc; }
cat > /tmp/c2l.py <<'PY'
import os, sys, time, numpy as np, torch
sys.path.insert(0, "pytorch-openpose_amd")
from src.body import Body
from src.hand import Hand
from src.weights import BENCH_OUT_SCALE, c5_out_scale, seeded_state_dict
body = Body(seeded_state_dict("body", 0, out_scale=BENCH_OUT_SCALE))
hand = Hand(seeded_state_dict("hand", 0))
body5 = Body(seeded_state_dict("body", 0, out_scale=c5_out_scale()), scale_search=(0.5, 1.0, 1.5, 2.0))
rng = np.random.default_rng(3)
img = rng.integers(0, 256, (368, 656, 3), dtype=np.uint8)
crop = rng.integers(0, 256, (368, 368, 3), dtype=np.uint8)
big = rng.integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
for _ in range(4): body(img); hand(crop); body5(big)
def med(fn, n):
    t = []
    for _ in range(n):
        t0 = time.perf_counter(); fn(); t.append(time.perf_counter() - t0)
    return np.median(t) * 1e3
print("small_ovh=%s C2 %.3f ms C3hand %.3f ms C5frame %.3f ms" % (os.environ.get("OPOSE_X6_SMALL_OVH", "1"),
      med(lambda: body(img), 40), med(lambda: hand(crop), 15), med(lambda: body5(big), 10)))
PY
timeout -k 10 120 python /tmp/c2l.py > /dev/null || exit 1
for o in 1 0 1 0; do
  export OPOSE_X6_SMALL_OVH=$o
  timeout -k 10 150 python /tmp/c2l.py || exit 1
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/bo.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/bo.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']
print('   bench', round(d['value'],1), round(d['ms_per_step'],3), {k: s[k] for k in ('conv1x1','conv3x3','conv7x7') if k in s})"
done
