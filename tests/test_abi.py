"""CPU-side checks of the C-ABI boundary: the library loads, exports every symbol include/*.h
declares, and validates arguments before touching the device."""
import ctypes
import subprocess

import pytest


def test_library_exports_every_declared_symbol(mfhe):
    names = mfhe.declared_symbols()
    assert "mfhe_ntt_fwd" in names and "mfhe_crt_compose" in names
    missing = [n for n in names if not hasattr(mfhe.lib, n)]
    assert not missing, f"declared but not exported: {missing}"
    out = subprocess.run(["nm", "-D", "--defined-only", str(mfhe.LIB_PATH)], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert set(names) <= exported


def test_version_and_error_channel(mfhe):
    assert b"gfx950" in mfhe.lib.mfhe_version()
    h = ctypes.c_void_p()
    arr = (ctypes.c_uint64 * 1)(15)   # not prime
    rc = mfhe.lib.mfhe_ctx_create(arr, 1, 6, mfhe.CONV_PHANTOM, 2.0 ** 35, ctypes.byref(h))
    assert rc == mfhe.EINVAL
    assert b"not a prime" in mfhe.lib.mfhe_last_error()
    rc = mfhe.lib.mfhe_ctx_create(arr, 1, 6, mfhe.CONV_PHANTOM, 2.0 ** 35, None)
    assert rc == mfhe.EINVAL
    arr2 = (ctypes.c_uint64 * 1)(17592186435073)
    rc = mfhe.lib.mfhe_ctx_create(arr2, 1, 25, mfhe.CONV_PHANTOM, 2.0 ** 35, ctypes.byref(h))
    assert rc == mfhe.EINVAL   # log_n out of range
    assert mfhe.lib.mfhe_ntt_fwd(None, None, 1, 0, 1, None) == mfhe.EINVAL


def test_no_cpu_fallback_in_product():
    """The product path must not import or link the oracle."""
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent / "matrix-fhe-gpu_amd"
    for p in list(root.rglob("*.py")) + list(root.rglob("*.hip")) + list(root.rglob("*.cpp")) + list(root.rglob("*.hpp")):
        text = p.read_text()
        assert "liboracle" not in text and "mfhe_oracle" not in text and "import oracle" not in text, p
