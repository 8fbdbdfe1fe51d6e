import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "pytorch-openpose_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def golden_image(d):
    """The input image of a body_e2e fixture: stored, or regenerated from its seed (C2-size
    fixtures keep only the seed and a checksum; oracle/gen_golden.py e2e_c2)."""
    import numpy as np
    if "img" in d:
        return d["img"]
    img = np.random.default_rng(int(d["img_seed"])).integers(0, 256, size=tuple(d["img_hw"]) + (3,), dtype=np.uint8)
    assert int(img.astype(np.int64).sum()) == int(d["img_sum"])
    return img


# lines a passing test wants in the run's log (pytest captures their prints): written in the
# terminal summary, e.g. the moved-keypoint count of every end-to-end fixture
REPORT_LINES = []


def report(line: str):
    REPORT_LINES.append(line)


def pytest_terminal_summary(terminalreporter):
    if REPORT_LINES:
        terminalreporter.section("libopose parity report")
        for line in REPORT_LINES:
            terminalreporter.write_line(line)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libopose.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
