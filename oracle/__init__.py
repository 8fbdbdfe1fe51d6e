"""ORACLE — test infrastructure only.

CPU restatement of the reference's OpenPose Body/Hand inference path
(hitmaxiang/pytorch-openpose `src/`).  Only `tests/`, `__graft_entry__.smoke()`
and `bench.py`'s `cpu_baseline` leg may import this package, and only as the
checker / the timed CPU baseline — never as the product path.

Modules
-------
cv_resize   OpenCV INTER_CUBIC restatement (uint8 fixed-point + float32 paths).
            Parity *unpinned* against real OpenCV (cv2 is absent here); pinned
            only by self-consistency — see DESIGN.md §Oracle.
network     torch-CPU conv graph restating `src/model.py` (pinned by golden
            outputs of the imported reference model).
body_post   NumPy/SciPy restatement of `src/body.py:32-212` (pinned by golden
            outputs of the imported reference `Body.__call__`).
hand_post   NumPy/SciPy restatement of `src/hand.py:32-75` (pinned likewise).
"""
