"""ctypes binding of libopose.so (the C ABI declared in include/opose.h).

This is the only way the package computes anything: there is no CPU fallback.  If the
shared library is missing or fails to load, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OPOSE_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libopose.so"))

OPOSE_OK = 0
OPOSE_E_ARG, OPOSE_E_SHAPE, OPOSE_E_HIP, OPOSE_E_WEIGHTS, OPOSE_E_CAPACITY, OPOSE_E_ASSEMBLY = -1, -2, -3, -4, -5, -6
OPOSE_E_TIMEOUT = -7
NET_BODY, NET_HAND = 0, 1
IN_DEVICE, OUT_DEVICE, PIPELINE, PIPELINE_DEFER = 1, 2, 4, 8
MAX_SCALES = 8


class Params(C.Structure):
    _fields_ = [("n_scales", C.c_int), ("scales", C.c_double * MAX_SCALES), ("boxsize", C.c_double),
                ("stride", C.c_int), ("pad_value", C.c_int), ("thre1", C.c_double), ("thre2", C.c_double),
                ("thre_hand", C.c_double)]


# int (*opose_halo_fn)(void* user, size_t bytes, void* stream)
HALO_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_size_t, C.c_void_p)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libopose.so not found at {LIB_PATH}: build it with `make -C pytorch-openpose_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    P, I, D, S = C.c_void_p, C.c_int, C.c_double, C.c_size_t
    sig = {
        "opose_default_params": (None, [I, C.POINTER(Params)]),
        "opose_create": (I, [I, C.POINTER(P)]),
        "opose_destroy": (None, [P]),
        "opose_last_error": (C.c_char_p, [P]),
        "opose_set_stream": (I, [P, P]),
        "opose_wait_stream": (I, [P, P]),
        "opose_signal_stream": (I, [P, P]),
        "opose_signal_input": (I, [P, P]),
        "opose_get_stream": (P, [P]),
        "opose_synchronize": (I, [P]),
        "opose_flush": (I, [P]),
        "opose_set_capacity": (I, [P, I, I]),
        "opose_body_record_bytes": (S, [P]),
        "opose_load_weights": (I, [P, I, C.POINTER(P), P, I]),
        "opose_body_forward": (I, [P, P, I, I, I, P, P, I]),
        "opose_hand_forward": (I, [P, P, I, I, I, P, I]),
        "opose_hand_forward_pyramid": (I, [P, I, C.POINTER(P), P, P, P, C.POINTER(P), I]),
        "opose_body_infer": (I, [P, P, I, I, I, C.c_int64, C.c_int64, C.POINTER(Params), P, I]),
        "opose_body_post": (I, [P, P, I, I, I, I, I, I, I, C.POINTER(Params), P, I]),
        "opose_body_scale_geom": (I, [I, I, C.POINTER(Params), I, P]),
        "opose_body_scale_maps": (I, [P, P, I, I, I, C.c_int64, C.c_int64, C.POINTER(Params), I, P, I]),
        "opose_body_post_scales": (I, [P, C.POINTER(P), P, P, P, P, I, I, I, I, C.POINTER(Params), P, I]),
        "opose_body_band_halo_bytes": (S, [I]),
        "opose_rccl_unique_id": (I, [P, S]),
        "opose_rccl_init": (I, [P, P, I, I]),
        "opose_rccl_abort": (I, [P]),
        "opose_rccl_wait": (I, [P, I]),
        "opose_set_band_peers": (I, [P, I, I]),
        "opose_body_band_maps": (I, [P, P, I, I, C.c_int64, C.POINTER(Params), I, I, I, P, HALO_FN, P, P, S, I]),
        "opose_hand_infer": (I, [P, P, I, I, I, C.c_int64, C.c_int64, C.POINTER(Params), P, P, I]),
        "opose_hand_post": (I, [P, C.POINTER(P), P, P, P, P, I, I, I, I, C.POINTER(Params), P, P, I]),
        "opose_hand_infer_crops": (I, [P, C.POINTER(P), P, P, I, C.POINTER(Params), P, P, I]),
        "opose_batch_body_infer": (I, [P, P, I, I, I, C.c_int64, C.c_int64, C.POINTER(Params), P, I]),
        "opose_batch_body_post": (I, [P, P, I, I, I, I, I, I, I, C.POINTER(Params), P, I]),
        "opose_batch_hand_infer": (I, [P, P, I, I, I, C.c_int64, C.c_int64, C.POINTER(Params), P, P, I]),
        "opose_batch_hand_post": (I, [P, P, I, I, I, C.POINTER(Params), P, P, I]),
        "opose_profile_enable": (I, [P, I]),
        "opose_profile_reset": (I, [P]),
        "opose_profile_read": (I, [P, C.c_char_p, S]),
        "opose_debug_conv": (I, [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, P]),
        "opose_debug_preprocess": (I, [P, P, I, I, D, I, P, P]),
        "opose_debug_conv_time": (I, [P, I, I, I, I, I, I, I, I, I, I, I, I, P]),
        "opose_debug_conv_x6": (I, [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P]),
        "opose_debug_conv_x6_time": (I, [P, I, I, I, I, I, I, I, I, I, I, I, P]),
        "opose_debug_heat": (I, [P, P, I, I, I, I, I, I, P, P]),
        "opose_debug_hand_label": (I, [P, P, I, I, I, D, P, P]),
    }
    for name, (res, args) in sig.items():
        if "OPOSE_LIB" in os.environ and not hasattr(lib, name):
            continue  # an older build picked for a same-box A/B may predate later entry points
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _ = D
    return lib


lib = _load()

EXPORTED = ["opose_default_params", "opose_create", "opose_destroy", "opose_last_error", "opose_set_stream",
            "opose_wait_stream", "opose_signal_stream", "opose_signal_input",
            "opose_get_stream", "opose_synchronize", "opose_flush", "opose_set_capacity", "opose_body_record_bytes",
            "opose_load_weights", "opose_body_forward", "opose_hand_forward", "opose_hand_forward_pyramid",
            "opose_body_infer",
            "opose_body_post", "opose_body_scale_geom", "opose_body_scale_maps",
            "opose_body_post_scales", "opose_body_band_halo_bytes", "opose_body_band_maps", "opose_rccl_unique_id", "opose_rccl_init", "opose_rccl_abort", "opose_rccl_wait", "opose_set_band_peers", "opose_batch_body_infer", "opose_batch_body_post", "opose_batch_hand_infer", "opose_batch_hand_post", "opose_hand_infer", "opose_hand_infer_crops", "opose_hand_post", "opose_profile_enable",
            "opose_profile_reset", "opose_profile_read", "opose_debug_conv", "opose_debug_conv_time", "opose_debug_conv_x6", "opose_debug_conv_x6_time", "opose_debug_preprocess",
            "opose_debug_heat", "opose_debug_hand_label"]


class OposeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libopose error {code}: {msg}")
        self.code = code


def default_params(net: int, **kw) -> Params:
    p = Params()
    lib.opose_default_params(net, C.byref(p))
    if "scale_search" in kw and kw["scale_search"] is not None:
        ss = list(kw.pop("scale_search"))
        if not 1 <= len(ss) <= MAX_SCALES:
            raise ValueError("scale_search must have 1..8 entries")
        p.n_scales = len(ss)
        for i, s in enumerate(ss):
            p.scales[i] = float(s)
    for k, v in kw.items():
        if v is not None:
            setattr(p, k, v)
    return p


def _ptr(a) -> int:
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())  # torch tensor


class Handle:
    """One device, one stream, weights + workspace (opose_t*)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        rc = lib.opose_create(int(device), C.byref(h))
        if rc != OPOSE_OK:
            raise OposeError(rc, "opose_create failed (no usable HIP device?)")
        self.h = h
        self.device = device
        # The handle runs on the library's own stream until the first device-tensor call
        # (wait_torch / signal_torch / hold): numpy-only callers never import torch or touch its
        # HIP context.  From then on the handle's stream is a torch pool stream (torch never
        # destroys those), so tensors whose last use is queued there (Handle.hold ->
        # record_stream) can be freed at any time, even after this handle is gone.  Torch hands
        # out its 32 pool streams per device round-robin: an unrelated torch.cuda.Stream() may be
        # the same HIP stream.  That only serialises the two users; opose_wait_stream /
        # opose_signal_stream order the library's streams correctly when a caller's stream is
        # the handle's own (tests/test_gpu_streams.py).
        self._torch_stream_obj = None

    def close(self):
        if getattr(self, "h", None):
            lib.opose_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int):
        if rc != OPOSE_OK:
            raise OposeError(rc, (lib.opose_last_error(self.h) or b"").decode())
        return rc

    # ---- configuration
    def set_capacity(self, peaks_per_part: int, max_people: int):
        self.check(lib.opose_set_capacity(self.h, peaks_per_part, max_people))

    def record_bytes(self) -> int:
        return int(lib.opose_body_record_bytes(self.h))

    def set_stream(self, stream_ptr: int | None):
        self.check(lib.opose_set_stream(self.h, stream_ptr or None))

    def stream(self) -> int:
        return lib.opose_get_stream(self.h) or 0

    def torch_stream(self):
        """The handle's stream as a torch.cuda.Stream (adopting a torch pool stream first): what
        consumers of pipelined outputs order themselves on."""
        self._adopt_torch_stream()
        return self._torch_stream_obj

    def synchronize(self):
        self.check(lib.opose_synchronize(self.h))

    def flush(self):
        """Enqueue a post-network part deferred by a pipeline="defer" call (OPOSE_PIPELINE_DEFER):
        afterwards the last call's records are complete in the handle's stream order."""
        self.check(lib.opose_flush(self.h))

    # ---- RCCL for row-band halo exchanges (opose_body_band_maps with the library's exchange)
    @staticmethod
    def rccl_unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        rc = lib.opose_rccl_unique_id(buf, 128)
        if rc != OPOSE_OK:
            raise OposeError(rc, "ncclGetUniqueId failed")
        return bytes(buf)

    def rccl_init(self, uid: bytes, rank: int, nranks: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid[:128])
        self.check(lib.opose_rccl_init(self.h, buf, int(rank), int(nranks)))

    def rccl_abort(self):
        """ncclCommAbort on the band communicator: this rank's own queued halo send / recv exit.
        It does not reach the neighbours' queued kernels; they bound their wait with rccl_wait."""
        self.check(lib.opose_rccl_abort(self.h))

    def rccl_wait(self, timeout_s: float):
        """Wait for the handle's stream (the RCCL halo exchanges of band_maps) for at most
        timeout_s.  A neighbour that failed, or an asynchronous RCCL error, makes the library abort
        this rank's communicator so its queued send / recv exit: TimeoutError / OposeError."""
        rc = lib.opose_rccl_wait(self.h, max(0, int(timeout_s * 1000)))
        if rc == OPOSE_E_TIMEOUT:
            raise TimeoutError((lib.opose_last_error(self.h) or b"").decode())
        self.check(rc)

    def set_band_peers(self, up, dn):
        self.check(lib.opose_set_band_peers(self.h, -1 if up is None else int(up), -1 if dn is None else int(dn)))

    # ---- ordering against torch's current stream (every device-tensor entry point)
    def _adopt_torch_stream(self):
        if self._torch_stream_obj is None:
            import torch
            self._torch_stream_obj = torch.cuda.Stream(device=torch.device("cuda", self.device))
            self.set_stream(self._torch_stream_obj.cuda_stream)  # ordered after the library's own stream

    def _torch_stream(self):
        import torch
        self._adopt_torch_stream()
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream or None)

    def wait_torch(self):
        """The handle's next work starts after everything queued on torch's current stream."""
        self.check(lib.opose_wait_stream(self.h, self._torch_stream()))

    def signal_torch(self):
        """Torch's current stream continues after everything queued on the handle: outputs are
        complete for torch consumers and the inputs the handle read may be freed/reused."""
        self.check(lib.opose_signal_stream(self.h, self._torch_stream()))

    def signal_input(self, stream=None):
        """Work queued on `stream` (a torch.cuda.Stream; default torch's current stream) from now on
        starts once the handle has read the device inputs of every call so far: after pipelined
        calls, the end of the last call's network part (opose_signal_input)."""
        import torch
        self._adopt_torch_stream()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.check(lib.opose_signal_input(self.h, C.c_void_p(st.cuda_stream or None)))

    def hold(self, *tensors):
        """Keep the caching allocator from reusing these tensors' memory until the handle's
        stream passes this point (asynchronous calls whose outputs stay on the handle's stream)."""
        self._adopt_torch_stream()
        st = self._torch_stream_obj
        if st.cuda_stream != self.stream():
            raise RuntimeError("Handle.hold needs the handle on its torch pool stream (set_stream changed it)")
        for t in tensors:
            t.record_stream(st)

    # ---- weights
    def load_weights(self, net: int, tensors):
        """tensors: list of float32 C-contiguous numpy arrays in reference state_dict order."""
        arrs = [np.ascontiguousarray(t, dtype=np.float32) for t in tensors]
        ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        shapes = np.ones((len(arrs), 4), np.int64)
        for i, a in enumerate(arrs):
            shapes[i, :a.ndim] = a.shape
        self.check(lib.opose_load_weights(self.h, net, ptrs, shapes.ctypes.data, len(arrs)))

    # ---- profiling
    def profile(self, enable: bool):
        self.check(lib.opose_profile_enable(self.h, int(enable)))

    def profile_reset(self):
        self.check(lib.opose_profile_reset(self.h))

    def profile_read(self) -> dict:
        import json
        buf = C.create_string_buffer(1 << 20)
        self.check(lib.opose_profile_read(self.h, buf, len(buf)))
        return json.loads(buf.value.decode())


def record_bytes(peaks_per_part: int, max_people: int) -> int:
    return 16 + 32 * 18 * peaks_per_part + 160 * max_people


def encode_record(candidate, subset, peaks_per_part: int, max_people: int, status: int = 0) -> np.ndarray:
    """Inverse of decode_record (host-side; used by tests and tools)."""
    rec = np.zeros(record_bytes(peaks_per_part, max_people), np.uint8)
    cand = np.asarray(candidate, np.float64).reshape(-1, 4)
    sub = np.asarray(subset, np.float64).reshape(-1, 20)
    if len(cand) > 18 * peaks_per_part or len(sub) > max_people:
        raise ValueError("record capacity exceeded")
    rec[:16].view(np.int32)[:3] = (status, len(cand), len(sub))
    rec[16:16 + 32 * len(cand)].view(np.float64)[:] = cand.ravel()
    off = 16 + 32 * 18 * peaks_per_part
    rec[off:off + 160 * len(sub)].view(np.float64)[:] = sub.ravel()
    return rec


def decode_record(rec: np.ndarray, peaks_per_part: int, max_people: int):
    """One Body record (uint8 view) -> (status, candidate, subset) in the reference's dtypes."""
    hdr = rec[:16].view(np.int32)
    status, n_cand, n_people = int(hdr[0]), int(hdr[1]), int(hdr[2])
    cap_c = 18 * peaks_per_part
    cand = rec[16:16 + 32 * cap_c].view(np.float64).reshape(cap_c, 4)[:n_cand].copy()
    off = 16 + 32 * cap_c
    sub = rec[off:off + 160 * max_people].view(np.float64).reshape(max_people, 20)[:n_people].copy()
    if n_cand == 0:
        cand = np.array([])          # np.array([]) in the reference when no peak exists (src/body.py:160)
    if n_people == 0:
        sub = -1 * np.ones((0, 20))  # src/body.py:159
    return status, cand, sub
