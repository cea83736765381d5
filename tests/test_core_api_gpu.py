"""The reference's own include/core + phantom C++ API, relinked against libmfhe.so (tests/cpp/).

Each program restates a reference test (test_custom_ntt_roundtrip.cu, phantom_ntt_roundtrip.cu,
test_encode_decode_loop.cu, test_wcrt_roundtrip.cu, src/main.cu) with host-side checks and exits
non-zero on failure.  They run as child processes, one at a time.
"""
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
CPP = Path(__file__).resolve().parent / "cpp"


def _run(name, *args, timeout=300):
    exe = CPP / name
    if not exe.exists():
        subprocess.run(["make", "-C", str(CPP), name], check=True, capture_output=True)
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=timeout)
    print(r.stdout[-4000:])
    assert r.returncode == 0, f"{name} failed ({r.returncode}):\n{r.stdout[-4000:]}\n{r.stderr[-2000:]}"
    return r.stdout


def test_core_ntt_api():
    out = _run("core_ntt_test")
    assert "[PASS]" in out


def test_core_he_api():
    out = _run("core_he_test")
    assert "[PASS]" in out


def test_pipeline_main_reference_flow():
    """src/main.cu: encode -> keygen -> encrypt_pair -> decrypt_and_decode, max error < 1e-4."""
    out = _run("pipeline_main", "1")
    assert "[SUCCESS]" in out
