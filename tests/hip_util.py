"""Tiny HIP runtime helpers for tests (raw device pointer <-> numpy)."""
import ctypes

import numpy as np

_hip = ctypes.CDLL("libamdhip64.so")
_hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
_hip.hipMemcpy.restype = ctypes.c_int
_hip.hipDeviceSynchronize.restype = ctypes.c_int


def d2h(dst: np.ndarray, src_ptr: int) -> np.ndarray:
    assert _hip.hipDeviceSynchronize() == 0
    rc = _hip.hipMemcpy(dst.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(src_ptr), dst.nbytes, 2)
    assert rc == 0, f"hipMemcpy D2H failed: {rc}"
    return dst
