"""mfhe -- Python host layer over libmfhe.so (include/mfhe.h), the MI355X backend for the
Matrix-FHE-GPU hot path (batched NTT/INTT, wide RNS CRT encode/decode).

The reference exposes this path through C++ (include/core/*.cuh) and phantom-fhe; this
module mirrors that surface for tests and benchmarks.  PyTorch is used only for device
memory and streams: every tensor is handed to the native library as a raw pointer.
There is no CPU or PyTorch fallback -- if libmfhe.so is missing or fails to load, import
raises.
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

_PKG_DIR = Path(__file__).resolve().parent.parent          # matrix-fhe-gpu_amd/
REPO_ROOT = _PKG_DIR.parent
# MFHE_LIB: load a tuning-variant build instead (tools only; the product path is libmfhe.so)
LIB_PATH = Path(os.environ["MFHE_LIB"]) if os.environ.get("MFHE_LIB") else _PKG_DIR / "libmfhe.so"
HEADER = REPO_ROOT / "include" / "mfhe.h"

OK, EINVAL, EUNSUPPORTED, EHIP, ENOMEM, ENOTREADY = 0, 1, 2, 3, 4, 5
CONV_PHANTOM, CONV_GL, CONV_WCRT = 1, 2, 4
ARITH_AUTO, ARITH_F64, ARITH_U64 = 0, 1, 2
OPT_NTT_CHUNK_BYTES, OPT_NTT_PLAN, OPT_CRT_WORDS, OPT_NTT_WG_PER_CU, OPT_NTT_PREFETCH = 1, 2, 3, 4, 5
OPT_NTT_FUSED, OPT_WCRT_MFMA = 6, 9   # OPT_NTT_FUSED: removed in r04, only 0 accepted
OPT_CGEMM_MFMA, OPT_HE_FUSED, OPT_TRACE_SPLIT = 10, 11, 12
XCHG_ALLGATHER, XCHG_ALLTOALL = 0, 1
RECOMBINE_ROWS_GLOBAL = 1
RECOMBINE_EXCHANGE_ONLY = 2     # measurement: exchanges only, composes skipped (out untouched)
RECOMBINE_AFTER_PREV = 4        # the shard was complete when the previous chunked call on the comm was entered
RECOMBINE_AGREE = 8             # end with an all-rank status agreement (host wait)
RECOMBINE_COMPOSE_ONLY = 16     # measurement: composes only, out of the receive halves' last exchanged chunks
RECOMBINE_SELF_EXCHANGE = 32    # test hook: world 1 runs the exchange pipeline (RCCL self-exchange) anyway
RECOMBINE_DEBUG_FAIL = 256      # test hook: the compose of chunk 1 (or 0) fails
OPT_NTT_PACK = 13
OPT_WCRT_PIPE = 14
OPT_NTT_PLAN_EFFECTIVE = 15   # read-only: 4 pipelined single pass (2^14 FP64), 1 single pass, 2 two passes
OPT_NTT_U60 = 17              # U64 NTTs with every modulus < 2^60: 1 = lazy U60 schedules (default), 0 = Harvey
OPT_HE_STREAMS = 18           # encode / encrypt_pair / decrypt_and_decode re/im chains: 3 = encode pairs + decode side stream (default), 2 = pairs, 1 = side stream, 0 = one stream
OPT_ENC_A_DIRECT = 19         # encrypt (fused ring): 1 = the GEMM writes a into both ciphertexts (default), 0 = ring kernel copies it
OPT_ENC_E_SMALL = 21          # encrypt: 1 = the noise's W-CRT as the dense product with its one digit (default), 0 = factored
OPT_DEC_MM = 20               # removed in r06 (the decrypt's ring product on the matrix cores): only 0 accepted; was FP64 X-NTT rows (default)
COMM_ID_BYTES = 128

#: reference parameters (include/core/config.h:7-52)
RNS_MODULI = [
    17592186435073, 17182765057, 17184541441, 17186120449, 17186515201, 17186909953,
    17188883713, 17190462721, 17190857473, 17191844353, 17192831233,
]
P_MODULI = [18014398515156481, 549757491457, 549759662593]
MATRIX_N = 64
BATCH_SIZE = 512
BATCH_PRIME_P = 771
SCALING_FACTOR = 2.0 ** 35


class MfheError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mfhe error {code}: {msg}")
        self.code = code


def _load() -> ctypes.CDLL:
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} not built; run `make -C {_PKG_DIR}` (or __graft_entry__.build())")
    return ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)


lib = _load()

_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t


class CtxInfo(ctypes.Structure):
    _fields_ = [
        ("num_limbs", ctypes.c_int), ("log_n", ctypes.c_int), ("crt_words", ctypes.c_int),
        ("arith", ctypes.c_int), ("conventions", ctypes.c_int), ("phi", ctypes.c_int),
        ("delta", ctypes.c_double),
    ]


def _sig(name, argtypes, restype=ctypes.c_int):
    f = getattr(lib, name)
    f.argtypes = argtypes
    f.restype = restype
    return f


_sig("mfhe_ctx_create", [_u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.POINTER(_vp)])
_sig("mfhe_ctx_destroy", [_vp])
_sig("mfhe_ctx_get_info", [_vp, ctypes.POINTER(CtxInfo)])
_sig("mfhe_ctx_set_arith", [_vp, ctypes.c_int])
_sig("mfhe_ctx_get_moduli", [_vp, _u64p, ctypes.c_int])
_sig("mfhe_ctx_set_option", [_vp, ctypes.c_int, ctypes.c_int64])
_sig("mfhe_ctx_get_option", [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)])
for _n in ("mfhe_ntt_fwd", "mfhe_ntt_inv", "mfhe_gl_ntt_fwd", "mfhe_gl_ntt_inv", "mfhe_cyclic_ntt_fwd",
           "mfhe_cyclic_ntt_inv"):
    _sig(_n, [_vp, _vp, _sz, ctypes.c_int, ctypes.c_int, _vp])
_sig("mfhe_gl_perm", [_vp, _vp, _vp, _sz, ctypes.c_int, ctypes.c_int, _vp])
_sig("mfhe_ntt_tables", [_vp] + [ctypes.POINTER(_vp)] * 6)
_sig("mfhe_ntt_dmodulus", [_vp, ctypes.POINTER(_vp)])
_sig("mfhe_fnwt_1d", [_vp, _vp, _vp, _vp, _sz, _sz, _sz, _sz, _vp])
_sig("mfhe_inwt_1d", [_vp, _vp, _vp, _vp, _vp, _vp, _sz, _sz, _sz, _sz, _vp])
_sig("mfhe_rns_decompose", [_vp, _vp, _sz, _sz, _sz, _vp, _vp])
_sig("mfhe_crt_compose", [_vp, _vp, _sz, _sz, _vp, _vp, _vp])
_sig("mfhe_crt_to_f64", [_vp, _vp, _vp, _sz, _vp, _sz, _vp])
_sig("mfhe_crt_compose_i64", [_vp, _vp, _sz, _sz, _vp, _vp])
_sig("mfhe_crt_compose_f64", [_vp, _vp, _sz, _sz, _vp, _sz, _vp])
_sig("mfhe_crt_compose_f64_sharded", [_vp, _vp, ctypes.c_int, _sz, _sz, _sz, _vp, _sz, _vp])
for _n in ("mfhe_wcrt_fwd", "mfhe_wcrt_inv", "mfhe_wcrt_fwd_vector", "mfhe_wcrt_fwd_centered",
           "mfhe_wcrt_inv_centered", "mfhe_wdft_fwd", "mfhe_wdft_inv", "mfhe_matrix_to_poly", "mfhe_poly_to_matrix",
           "mfhe_keygen"):
    _sig(_n, [_vp, _vp, _vp, _vp] if _n != "mfhe_keygen" else [_vp, _vp, _vp])
_sig("mfhe_xy_idft", [_vp, _vp, _vp, _sz, _vp])
_sig("mfhe_xy_dft", [_vp, _vp, _vp, _sz, _vp])
_sig("mfhe_wdft_fwd_pair_i64", [_vp] * 6)
_sig("mfhe_wdft_inv_pair", [_vp] * 6)
_sig("mfhe_ct_add", [_vp] * 5)
_sig("mfhe_ct_mul_tensor", [_vp] * 7)
_sig("mfhe_trace_map_bprime", [_vp] * 5 + [ctypes.c_int, ctypes.c_int, _sz, _vp])
_sig("mfhe_trace_gemm", [_vp] * 7 + [ctypes.c_int, ctypes.c_int, _sz, _vp])
_sig("mfhe_trace_rescale", [_vp] * 3 + [ctypes.c_int, ctypes.c_int, _sz, _u64p, _vp])
_sig("mfhe_trace_product", [_vp] * 7 + [ctypes.c_int, ctypes.c_int, _sz, _u64p, _vp])
_sig("mfhe_ctx_reserve_workspace", [_vp])
_sig("mfhe_encode", [_vp, _vp, _vp, _vp, _vp])
_sig("mfhe_decode", [_vp, _vp, _vp, _vp, _vp])
_sig("mfhe_encrypt", [_vp, _vp, _vp, _vp, _vp])
_sig("mfhe_encrypt_pair", [_vp, _vp, _vp, _vp, _vp, _vp, _vp])
_sig("mfhe_decrypt_to_eval", [_vp, _vp, _vp, _vp, _vp])
_sig("mfhe_decrypt_and_decode", [_vp, _vp, _vp, _vp, _vp, _vp])
_sig("mfhe_comm_unique_id", [_vp])
_sig("mfhe_comm_init", [_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp)])
_sig("mfhe_comm_wrap", [_vp, ctypes.POINTER(_vp)])
_sig("mfhe_comm_destroy", [_vp])
_sig("mfhe_comm_info", [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)])
_sig("mfhe_allgather_limbs", [_vp, _vp, _sz, _vp, _vp])
_sig("mfhe_crt_recombine_sharded", [_vp, _vp, ctypes.c_int, _vp, _sz, _sz, _vp, _sz, _vp])
_sig("mfhe_crt_recombine_reserve", [_vp, _vp, ctypes.c_int, _sz, _sz])
_sig("mfhe_crt_recombine_chunked", [_vp, _vp, ctypes.c_int, _vp, _sz, _sz, _sz, _vp, _sz, ctypes.c_int, _vp])
_sig("mfhe_crt_recombine_chunked_reserve", [_vp, _vp, ctypes.c_int, _sz, _sz])
_sig("mfhe_ctx_set_limb_shard", [_vp, ctypes.c_int, ctypes.c_int])
_sig("mfhe_decode_sharded", [_vp, _vp, _vp, ctypes.c_int, _vp, _vp, _vp, _vp])
_sig("mfhe_decrypt_and_decode_sharded", [_vp, _vp, _vp, ctypes.c_int, _vp, _vp, _vp, _vp, _vp])
_sig("mfhe_last_error", [], ctypes.c_char_p)
_sig("mfhe_version", [], ctypes.c_char_p)


def declared_symbols(header: Path = None) -> list[str]:
    """Every function name declared in include/*.h (the C-ABI surface)."""
    hdrs = [header] if header else sorted((REPO_ROOT / "include").glob("*.h"))
    names = []
    for h in hdrs:
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names += re.findall(r"\b(mfhe_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def check(rc: int, what: str = "") -> None:
    if rc != OK:
        raise MfheError(rc, f"{what}: {lib.mfhe_last_error().decode()}")


_XCHG = {"allgather": XCHG_ALLGATHER, "alltoall": XCHG_ALLTOALL}


def _need(t, words, what):
    """Host-side size check before a raw pointer crosses the C ABI (an undersized tensor would otherwise be
    an out-of-bounds device access)."""
    if t.numel() * t.element_size() < 8 * words:
        raise ValueError(f"{what}: {t.numel()} elements of {t.element_size()} B < {words} words needed")


def _need_strided(t, count, stride, what):
    """An output written at t[i * stride], i < count: (count - 1) * stride + 1 words."""
    if stride < 1:
        raise ValueError(f"{what}: stride must be >= 1")
    _need(t, (count - 1) * stride + 1 if count else 0, what)


class _stdout_to_stderr:
    """RCCL's initialisation banner goes to fd 1; keep a caller's stdout (bench.py's one JSON line) clean."""

    def __enter__(self):
        import sys
        sys.stdout.flush()
        self._saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        os.dup2(self._saved, 1)
        os.close(self._saved)


class Comm:
    """An RCCL communicator owned by libmfhe (include/mfhe.h mfhe_comm_*): one per process/GPU.

    `Comm.create(rank, world, group)` makes rank 0 draw the unique id and broadcasts it over an existing
    torch.distributed process group (any backend) -- the side channel only; the data path is RCCL."""

    def __init__(self, handle, size, rank):
        self._h, self.size, self.rank = handle, size, rank

    @classmethod
    def from_id(cls, uid: bytes, world: int, rank: int) -> "Comm":
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        h = _vp()
        with _stdout_to_stderr():
            rc = lib.mfhe_comm_init(ctypes.addressof(buf), world, rank, ctypes.byref(h))
        check(rc, "comm_init")
        return cls(h, world, rank)

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
        with _stdout_to_stderr():
            rc = lib.mfhe_comm_unique_id(ctypes.addressof(buf))
        check(rc, "comm_unique_id")
        return bytes(buf)

    @classmethod
    def create(cls, group=None) -> "Comm":
        import torch
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = cls.unique_id() if rank == 0 else bytes(COMM_ID_BYTES)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        if dist.get_backend(group) == "nccl":
            t = t.cuda()
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return cls.from_id(bytes(t.cpu().tolist()), world, rank)

    def allgather_limbs(self, shard, recv, stream=None):
        _need(recv, shard.numel() * self.size, "recv")
        check(lib.mfhe_allgather_limbs(self._h, _ptr(shard), shard.numel(), _ptr(recv), _stream_ptr(stream)),
              "allgather_limbs")
        return recv

    def close(self):
        if self._h:
            check(lib.mfhe_comm_destroy(self._h), "comm_destroy")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _stream_ptr(stream) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _ptr(t) -> int:
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("mfhe operates on device tensors")
    if not t.is_contiguous():
        raise ValueError("mfhe needs contiguous tensors")
    return t.data_ptr()


class Context:
    """One parameter set + device tables (mfhe_ctx).  Mirrors init_he_backend /
    PhantomContext / Encoder table setup of the reference."""

    def __init__(self, moduli, log_n: int, conventions: int = CONV_PHANTOM, delta: float = SCALING_FACTOR):
        arr = (ctypes.c_uint64 * len(moduli))(*[int(m) for m in moduli])
        h = _vp()
        check(lib.mfhe_ctx_create(arr, len(moduli), int(log_n), int(conventions), float(delta), ctypes.byref(h)),
              "mfhe_ctx_create")
        self._h = h
        self.moduli = [int(m) for m in moduli]
        self.L = len(self.moduli)
        self.log_n = int(log_n)
        self.N = 1 << self.log_n
        self.delta = float(delta)
        info = self.info()
        self.crt_words = info.crt_words
        self.phi = info.phi

    @property
    def handle(self):
        return self._h

    def info(self) -> CtxInfo:
        inf = CtxInfo()
        check(lib.mfhe_ctx_get_info(self._h, ctypes.byref(inf)), "get_info")
        return inf

    def set_arith(self, arith: int) -> None:
        check(lib.mfhe_ctx_set_arith(self._h, arith), "set_arith")

    def set_option(self, opt: int, value: int) -> None:
        check(lib.mfhe_ctx_set_option(self._h, opt, int(value)), "set_option")

    def get_option(self, opt: int) -> int:
        v = ctypes.c_int64()
        check(lib.mfhe_ctx_get_option(self._h, opt, ctypes.byref(v)), "get_option")
        return v.value

    def close(self):
        if getattr(self, "_h", None):
            lib.mfhe_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- NTT ----
    def _ntt(self, fn, data, batch, start_limb, nlimbs, stream):
        nl = self.L - start_limb if nlimbs is None else nlimbs
        if batch is None:
            batch = data.numel() // (nl * self.N)
        if data.numel() < batch * nl * self.N:
            raise ValueError("tensor smaller than batch * nlimbs * N")
        check(fn(self._h, _ptr(data), batch, start_limb, nl, _stream_ptr(stream)), fn.__name__)
        return data

    def ntt_fwd(self, data, batch=None, start_limb=0, nlimbs=None, stream=None):
        return self._ntt(lib.mfhe_ntt_fwd, data, batch, start_limb, nlimbs, stream)

    def ntt_inv(self, data, batch=None, start_limb=0, nlimbs=None, stream=None):
        return self._ntt(lib.mfhe_ntt_inv, data, batch, start_limb, nlimbs, stream)

    def gl_ntt_fwd(self, data, batch=None, start_limb=0, nlimbs=None, stream=None):
        return self._ntt(lib.mfhe_gl_ntt_fwd, data, batch, start_limb, nlimbs, stream)

    def gl_ntt_inv(self, data, batch=None, start_limb=0, nlimbs=None, stream=None):
        return self._ntt(lib.mfhe_gl_ntt_inv, data, batch, start_limb, nlimbs, stream)

    def cyclic_ntt_fwd(self, data, batch=None, start_limb=0, nlimbs=None, stream=None):
        return self._ntt(lib.mfhe_cyclic_ntt_fwd, data, batch, start_limb, nlimbs, stream)

    def cyclic_ntt_inv(self, data, batch=None, start_limb=0, nlimbs=None, stream=None):
        return self._ntt(lib.mfhe_cyclic_ntt_inv, data, batch, start_limb, nlimbs, stream)

    def gl_perm(self, src, dst, batch, nlimbs=None, inverse=False, stream=None):
        nl = self.L if nlimbs is None else nlimbs
        check(lib.mfhe_gl_perm(self._h, _ptr(src), _ptr(dst), batch, nl, int(inverse), _stream_ptr(stream)), "gl_perm")
        return dst

    def ntt_tables(self):
        ps = [_vp() for _ in range(6)]
        check(lib.mfhe_ntt_tables(self._h, *[ctypes.byref(p) for p in ps]), "ntt_tables")
        dm = _vp()
        check(lib.mfhe_ntt_dmodulus(self._h, ctypes.byref(dm)), "ntt_dmodulus")
        return [p.value for p in ps] + [dm.value]

    # ---- wide CRT ----
    def rns_decompose(self, src, dst, npoly, ncoeff, in_stride=1, stream=None):
        check(lib.mfhe_rns_decompose(self._h, _ptr(src), in_stride, npoly, ncoeff, _ptr(dst), _stream_ptr(stream)),
              "rns_decompose")
        return dst

    def crt_compose(self, src, mag, neg, npoly, ncoeff, stream=None):
        check(lib.mfhe_crt_compose(self._h, _ptr(src), npoly, ncoeff, _ptr(mag), _ptr(neg), _stream_ptr(stream)),
              "crt_compose")

    def crt_compose_i64(self, src, out, npoly, ncoeff, stream=None):
        """Centred CRT value truncated to int64 (crt_compose_centerlift_kernel, encoder.cu:152-189)."""
        _need(src, npoly * self.L * ncoeff, "crt_compose_i64 src")
        _need(out, npoly * ncoeff, "crt_compose_i64 out")
        check(lib.mfhe_crt_compose_i64(self._h, _ptr(src), npoly, ncoeff, _ptr(out), _stream_ptr(stream)),
              "crt_compose_i64")
        return out

    def crt_to_f64(self, mag, neg, out, count, out_stride=1, stream=None):
        _need(mag, count * self.info().crt_words, "crt_to_f64 mag")
        _need_strided(out, count, out_stride, "crt_to_f64 out")
        check(lib.mfhe_crt_to_f64(self._h, _ptr(mag), _ptr(neg), count, _ptr(out), out_stride, _stream_ptr(stream)),
              "crt_to_f64")
        return out

    def crt_compose_f64(self, src, out, npoly, ncoeff, out_stride=1, stream=None):
        _need(src, npoly * self.L * ncoeff, "crt_compose_f64 src")
        _need_strided(out, npoly * ncoeff, out_stride, "crt_compose_f64 out")
        check(lib.mfhe_crt_compose_f64(self._h, _ptr(src), npoly, ncoeff, _ptr(out), out_stride, _stream_ptr(stream)),
              "crt_compose_f64")
        return out


    def crt_compose_f64_sharded(self, src, out, nshards, shard_stride, npoly, ncoeff, out_stride=1, stream=None,
                                src_offset=0):
        """Compose residue shards gathered from `nshards` GPUs in place (see include/mfhe.h)."""
        _need(src, src_offset + (nshards - 1) * shard_stride + npoly * (self.L // max(nshards, 1)) * ncoeff,
              "crt_compose_f64_sharded src")
        _need_strided(out, npoly * ncoeff, out_stride, "crt_compose_f64_sharded out")
        check(lib.mfhe_crt_compose_f64_sharded(self._h, _ptr(src) + 8 * src_offset, nshards, shard_stride, npoly,
                                               ncoeff, _ptr(out), out_stride, _stream_ptr(stream)),
              "crt_compose_f64_sharded")
        return out

    def crt_recombine_sharded(self, comm: "Comm", mode, shard, npoly, ncoeff, out, out_stride=1, stream=None):
        """RCCL exchange of this rank's [npoly][L/G][ncoeff] residue shard + compose of its polynomial slice
        (include/mfhe.h mfhe_crt_recombine_sharded); out: npoly/G * ncoeff f64."""
        m = _XCHG[mode] if isinstance(mode, str) else mode
        g = comm.size
        lg = self.info().num_limbs // g if g else 0
        _need(shard, npoly * lg * ncoeff, "shard")
        # the kernel writes out[i * out_stride] for i < npoly / G * ncoeff
        _need_strided(out, (npoly // g) * ncoeff if g else 0, out_stride, "out")
        check(lib.mfhe_crt_recombine_sharded(self._h, comm._h, m, _ptr(shard), npoly, ncoeff, _ptr(out), out_stride,
                                             _stream_ptr(stream)), "crt_recombine_sharded")
        return out

    def crt_recombine_reserve(self, comm: "Comm", mode, npoly, ncoeff):
        m = _XCHG[mode] if isinstance(mode, str) else mode
        check(lib.mfhe_crt_recombine_reserve(self._h, comm._h, m, npoly, ncoeff), "crt_recombine_reserve")

    def crt_recombine_chunked(self, comm: "Comm", mode, shard, npoly, ncoeff, chunk_polys, out, out_stride=1,
                              rows_global=False, stream=None, flags=0):
        """Chunked, pipelined RCCL recombine (include/mfhe.h mfhe_crt_recombine_chunked): exchange of chunk k + 1
        on the communicator's stream beside the compose of chunk k on `stream`.  out rows: owned_polys order
        (npoly/G rows), or the global poly index with rows_global (npoly rows, only this rank's written).
        flags: further MFHE_RECOMBINE_* bits (RECOMBINE_EXCHANGE_ONLY: out may be None)."""
        m = _XCHG[mode] if isinstance(mode, str) else mode
        g = comm.size
        lg = self.info().num_limbs // g if g else 0
        _need(shard, npoly * lg * ncoeff, "shard")
        rows = npoly if rows_global else (npoly // g if g else 0)
        if out is not None or not flags & RECOMBINE_EXCHANGE_ONLY:
            _need_strided(out, rows * ncoeff, out_stride, "out")
        check(lib.mfhe_crt_recombine_chunked(self._h, comm._h, m, _ptr(shard), npoly, ncoeff, chunk_polys,
                                             _ptr(out) if out is not None else None, out_stride,
                                             (RECOMBINE_ROWS_GLOBAL if rows_global else 0) | flags,
                                             _stream_ptr(stream)), "crt_recombine_chunked")
        return out

    def crt_recombine_chunked_reserve(self, comm: "Comm", mode, chunk_polys, ncoeff):
        m = _XCHG[mode] if isinstance(mode, str) else mode
        check(lib.mfhe_crt_recombine_chunked_reserve(self._h, comm._h, m, chunk_polys, ncoeff),
              "crt_recombine_chunked_reserve")

    # ---- W axis / encoder / pipelines (reference geometry, CONV_WCRT) ----
    def _call(self, name, *ptrs, stream=None):
        fn = getattr(lib, name)
        check(fn(self._h, *ptrs, _stream_ptr(stream)), name)

    # host-side sizes of the fixed-geometry buffers (phi = 512 W-lanes), checked before raw pointers cross
    def _mat(self):   # one matrix-major [phi][L][n*n] (or poly-major [phi*n][L][n]) residue array
        return 512 * self.L * self.N * self.N

    def _msg(self):   # one [phi][n*n] complex message, interleaved doubles
        return 2 * 512 * self.N * self.N

    def _sk(self):    # secret key [phi][L][n]
        return 512 * self.L * self.N

    def _sizes(self, what, *pairs):
        for t, words in pairs:
            _need(t, words, what)

    def wcrt_fwd(self, src, dst, stream=None):
        self._sizes("wcrt_fwd", (src, self._mat()), (dst, self._mat()))
        self._call("mfhe_wcrt_fwd", _ptr(src), _ptr(dst), stream=stream); return dst
    def wcrt_inv(self, src, dst, stream=None):
        self._sizes("wcrt_inv", (src, self._mat()), (dst, self._mat()))
        self._call("mfhe_wcrt_inv", _ptr(src), _ptr(dst), stream=stream); return dst
    def wcrt_fwd_vector(self, src, dst, stream=None):
        self._call("mfhe_wcrt_fwd_vector", _ptr(src), _ptr(dst), stream=stream); return dst
    def wcrt_fwd_centered(self, src, dst, stream=None):
        self._call("mfhe_wcrt_fwd_centered", _ptr(src), _ptr(dst), stream=stream); return dst
    def wcrt_inv_centered(self, src, dst, stream=None):
        self._call("mfhe_wcrt_inv_centered", _ptr(src), _ptr(dst), stream=stream); return dst
    def wdft_fwd(self, src, dst, stream=None): self._call("mfhe_wdft_fwd", _ptr(src), _ptr(dst), stream=stream); return dst
    def wdft_inv(self, src, dst, stream=None): self._call("mfhe_wdft_inv", _ptr(src), _ptr(dst), stream=stream); return dst
    def wdft_fwd_pair_i64(self, re, im, out_re, out_im, stream=None):
        self._call("mfhe_wdft_fwd_pair_i64", _ptr(re), _ptr(im), _ptr(out_re), _ptr(out_im), stream=stream)
    def wdft_inv_pair(self, re, im, out_re, out_im, stream=None):
        self._call("mfhe_wdft_inv_pair", _ptr(re), _ptr(im), _ptr(out_re), _ptr(out_im), stream=stream)
    def ct_add(self, ct1, ct2, res, stream=None):
        self._sizes("ct_add", *[(t, 2 * self._mat()) for t in (ct1, ct2, res)])
        self._call("mfhe_ct_add", _ptr(ct1), _ptr(ct2), _ptr(res), stream=stream); return res
    def ct_mul_tensor(self, ct1, ct2, d0, d1, d2, stream=None):
        self._sizes("ct_mul_tensor", (ct1, 2 * self._mat()), (ct2, 2 * self._mat()),
                    *[(t, self._mat()) for t in (d0, d1, d2)])
        self._call("mfhe_ct_mul_tensor", _ptr(ct1), _ptr(ct2), _ptr(d0), _ptr(d1), _ptr(d2), stream=stream)
    # ---- trace GEMM, planes [batch][nlimbs][n][n] (batched_trace.cu) ----
    @staticmethod
    def _trace_need(tensors, n, nlimbs, batch, what):
        """Every plane must hold batch * nlimbs * n * n int64/uint64 words (checked before raw pointers cross)."""
        import torch
        words = batch * nlimbs * n * n
        for t in tensors:
            if t.dtype not in (torch.int64, torch.uint64):
                raise ValueError(f"{what}: planes must be int64/uint64, got {t.dtype}")
            _need(t, words, what)

    def trace_map_bprime(self, b_re, b_im, bp_re, bp_im, n, nlimbs, batch, stream=None):
        self._trace_need((b_re, b_im, bp_re, bp_im), n, nlimbs, batch, "trace_map_bprime")
        check(lib.mfhe_trace_map_bprime(self._h, _ptr(b_re), _ptr(b_im), _ptr(bp_re), _ptr(bp_im), n, nlimbs, batch,
                                        _stream_ptr(stream)), "trace_map_bprime")
    def trace_gemm(self, a_re, a_im, bp_re, bp_im, c_re, c_im, n, nlimbs, batch, stream=None):
        self._trace_need((a_re, a_im, bp_re, bp_im, c_re, c_im), n, nlimbs, batch, "trace_gemm")
        check(lib.mfhe_trace_gemm(self._h, _ptr(a_re), _ptr(a_im), _ptr(bp_re), _ptr(bp_im), _ptr(c_re), _ptr(c_im),
                                  n, nlimbs, batch, _stream_ptr(stream)), "trace_gemm")
    def trace_rescale(self, c_re, c_im, n, nlimbs, batch, inv, stream=None):
        self._trace_need((c_re, c_im), n, nlimbs, batch, "trace_rescale")
        arr = (ctypes.c_uint64 * nlimbs)(*[int(v) for v in inv[:nlimbs]])
        check(lib.mfhe_trace_rescale(self._h, _ptr(c_re), _ptr(c_im), n, nlimbs, batch, arr, _stream_ptr(stream)),
              "trace_rescale")
    def trace_product(self, a_re, a_im, b_re, b_im, c_re, c_im, n, nlimbs, batch, inv=None, stream=None):
        self._trace_need((a_re, a_im, b_re, b_im, c_re, c_im), n, nlimbs, batch, "trace_product")
        arr = (ctypes.c_uint64 * nlimbs)(*[int(v) for v in inv[:nlimbs]]) if inv is not None else None
        check(lib.mfhe_trace_product(self._h, _ptr(a_re), _ptr(a_im), _ptr(b_re), _ptr(b_im), _ptr(c_re), _ptr(c_im),
                                     n, nlimbs, batch, arr, _stream_ptr(stream)), "trace_product")
    def xy_dft(self, src, dst, lanes, stream=None):
        check(lib.mfhe_xy_dft(self._h, _ptr(src), _ptr(dst), lanes, _stream_ptr(stream)), "xy_dft"); return dst
    def xy_idft(self, src, dst, lanes, stream=None):
        check(lib.mfhe_xy_idft(self._h, _ptr(src), _ptr(dst), lanes, _stream_ptr(stream)), "xy_idft"); return dst
    def matrix_to_poly(self, src, dst, stream=None):
        self._sizes("matrix_to_poly", (src, self._mat()), (dst, self._mat()))
        self._call("mfhe_matrix_to_poly", _ptr(src), _ptr(dst), stream=stream); return dst
    def poly_to_matrix(self, src, dst, stream=None):
        self._sizes("poly_to_matrix", (src, self._mat()), (dst, self._mat()))
        self._call("mfhe_poly_to_matrix", _ptr(src), _ptr(dst), stream=stream); return dst
    def reserve_workspace(self): check(lib.mfhe_ctx_reserve_workspace(self._h), "reserve_workspace")
    def encode(self, msg, out_re, out_im, stream=None):
        self._sizes("encode", (msg, self._msg()), (out_re, self._mat()), (out_im, self._mat()))
        self._call("mfhe_encode", _ptr(msg), _ptr(out_re), _ptr(out_im), stream=stream)
    def decode(self, ev_re, ev_im, msg, stream=None):
        self._sizes("decode", (ev_re, self._mat()), (ev_im, self._mat()), (msg, self._msg()))
        self._call("mfhe_decode", _ptr(ev_re), _ptr(ev_im), _ptr(msg), stream=stream); return msg
    def keygen(self, sk, stream=None):
        self._sizes("keygen", (sk, self._sk()))
        self._call("mfhe_keygen", _ptr(sk), stream=stream); return sk
    def encrypt(self, m, sk, ct, stream=None):
        self._sizes("encrypt", (m, self._mat()), (sk, self._sk()), (ct, 2 * self._mat()))
        self._call("mfhe_encrypt", _ptr(m), _ptr(sk), _ptr(ct), stream=stream)
    def encrypt_pair(self, m_re, m_im, sk, ct_re, ct_im, stream=None):
        self._sizes("encrypt_pair", (m_re, self._mat()), (m_im, self._mat()), (sk, self._sk()),
                    (ct_re, 2 * self._mat()), (ct_im, 2 * self._mat()))
        self._call("mfhe_encrypt_pair", _ptr(m_re), _ptr(m_im), _ptr(sk), _ptr(ct_re), _ptr(ct_im), stream=stream)
    def decrypt_to_eval(self, ct, sk, out, stream=None):
        self._sizes("decrypt_to_eval", (ct, 2 * self._mat()), (sk, self._sk()), (out, self._mat()))
        self._call("mfhe_decrypt_to_eval", _ptr(ct), _ptr(sk), _ptr(out), stream=stream); return out
    def decrypt_and_decode(self, ct_re, ct_im, sk, msg, stream=None):
        self._sizes("decrypt_and_decode", (ct_re, 2 * self._mat()), (ct_im, 2 * self._mat()), (sk, self._sk()),
                    (msg, self._msg()))
        self._call("mfhe_decrypt_and_decode", _ptr(ct_re), _ptr(ct_im), _ptr(sk), _ptr(msg), stream=stream); return msg

    # ---- residue sharding across GPUs (BASELINE C4, include/mfhe.h) ----
    def set_limb_shard(self, limb_base: int, limbs_total: int):
        """This context holds limbs [limb_base, limb_base + L) of a limbs_total-modulus parameter set."""
        check(lib.mfhe_ctx_set_limb_shard(self._h, limb_base, limbs_total), "set_limb_shard")

    def decode_sharded(self, ctx_all: "Context", comm: "Comm", mode, ev_re, ev_im, msg, stream=None):
        m = _XCHG[mode] if isinstance(mode, str) else mode
        self._sizes("decode_sharded", (ev_re, self._mat()), (ev_im, self._mat()), (msg, self._msg()))
        check(lib.mfhe_decode_sharded(self._h, ctx_all._h, comm._h, m, _ptr(ev_re), _ptr(ev_im), _ptr(msg),
                                      _stream_ptr(stream)), "decode_sharded")
        return msg

    def decrypt_and_decode_sharded(self, ctx_all: "Context", comm: "Comm", mode, ct_re, ct_im, sk, msg, stream=None):
        m = _XCHG[mode] if isinstance(mode, str) else mode
        self._sizes("decrypt_and_decode_sharded", (ct_re, 2 * self._mat()), (ct_im, 2 * self._mat()),
                    (sk, self._sk()), (msg, self._msg()))
        check(lib.mfhe_decrypt_and_decode_sharded(self._h, ctx_all._h, comm._h, m, _ptr(ct_re), _ptr(ct_im), _ptr(sk),
                                                  _ptr(msg), _stream_ptr(stream)), "decrypt_and_decode_sharded")
        return msg


def fnwt_1d(data, tw, tw_shoup, dmod, dim, coeff_modulus_size, start_modulus_idx=0, batch=1, stream=None):
    """phantom fnwt_1d (ntt/ntt_1d.cu) over raw table pointers; batch polys at once."""
    check(lib.mfhe_fnwt_1d(_ptr(data), tw, tw_shoup, dmod, dim, coeff_modulus_size, start_modulus_idx, batch,
                           _stream_ptr(stream)), "fnwt_1d")


def inwt_1d(data, itw, itw_shoup, dmod, scalar, scalar_shoup, dim, coeff_modulus_size, start_modulus_idx=0, batch=1,
            stream=None):
    check(lib.mfhe_inwt_1d(_ptr(data), itw, itw_shoup, dmod, scalar, scalar_shoup, dim, coeff_modulus_size,
                           start_modulus_idx, batch, _stream_ptr(stream)), "inwt_1d")


# ---- host/device array helpers (uint64 stored in int64 tensors) ----
def to_device_u64(arr, device="cuda"):
    import numpy as np
    import torch
    a = np.ascontiguousarray(arr, dtype=np.uint64)
    return torch.from_numpy(a.view(np.int64)).to(device)


def to_host_u64(t):
    import numpy as np
    return t.detach().cpu().numpy().view(np.uint64)
