"""Hand keypoints with the reference's call surface (hitmaxiang/pytorch-openpose src/hand.py).

Placeholder module: the hand network runs through libopose (`handpose_model`); the full
Hand() post-processing path lands with the hand kernels.
"""
from __future__ import annotations

from .model import handpose_model  # noqa: F401
