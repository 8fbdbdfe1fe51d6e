# Hand scales concurrent (default) vs sequential (OPOSE_SCALE_STREAMS=0): C3 Hand() latency on a
# 368x368 crop, one process per measurement.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
cat > /tmp/hl.py <<'PY'
import os, sys, time, numpy as np
sys.path.insert(0, "pytorch-openpose_amd")
from src.hand import Hand
from src.weights import seeded_state_dict
hand = Hand(seeded_state_dict("hand", 0))
crop = np.random.default_rng(5).integers(0, 256, (368, 368, 3), dtype=np.uint8)
for _ in range(3): hand(crop)
t = []
for _ in range(15):
    t0 = time.perf_counter(); hand(crop); t.append(time.perf_counter() - t0)
print("scale_streams=%s hand_ms %.3f" % (os.environ.get("OPOSE_SCALE_STREAMS", "1"), np.median(t) * 1e3))
PY
timeout -k 10 120 python /tmp/hl.py > /dev/null || exit 1
for rep in 1 2 3; do
  for s in 1 0; do OPOSE_SCALE_STREAMS=$s timeout -k 10 120 python /tmp/hl.py || exit 1; done
done
