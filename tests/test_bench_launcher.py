"""CPU: `bench.py --gpus N` starts N ranks itself (torch.distributed.run, before any GPU call)
and the gathered records come back in frame order; the --dry-run mode uses gloo and host
records, so the launcher and the gather run here without a GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ, **(env or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if env is None or k not in env:
            e.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=e,
                          capture_output=True, text=True, timeout=300)


def test_gpus_2_launches_two_ranks():
    out = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--batch", "4"])
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["frames_total"] == 2 * 4 * 2 and d["gathered_frames"] == 8


def test_gpus_8_launches_eight_ranks():
    """The driver's 8-GPU scaling run rehearsed: 8 gloo ranks x 32 frames, 256 records gathered
    in frame order (dry_run asserts the order on every rank), one line from rank 0."""
    out = _run(["--gpus", "8", "--dry-run", "--steps", "2", "--warmup", "1", "--batch", "32"])
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["gathered_frames"] == 256 and d["frames_total"] == 8 * 32 * 2


def test_world_size_must_match_gpus():
    out = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr
