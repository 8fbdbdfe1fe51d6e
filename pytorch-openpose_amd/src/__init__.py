"""MI355X-native drop-in for hitmaxiang/pytorch-openpose's `src` package (Body/Hand inference).

Put `pytorch-openpose_amd/` on sys.path and `from src.body import Body` exactly as with the
reference.  All compute runs in libopose.so (HIP, gfx950); importing fails loudly if it is
missing.
"""
