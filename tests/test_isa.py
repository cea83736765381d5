"""CPU check of the shipped code object: the forward column pass's counted waits (csrc/ntt_coldb.hpp).

ntt_col_db_kernel keeps the next tile's LDS-DMA in flight and waits for the current tile with
`s_waitcnt vmcnt(N)`, N = the vector-memory operations issued after that tile's DMA (16 stores + 8 DMAs).
That is only right while the compiled kernel issues exactly those: a spill (scratch_* ops), a split store or
an extra load in the loop would make the waits too loose and the butterflies would read LDS before the DMA
lands.  This test disassembles the gfx950 code object inside libmfhe.so and pins the kernel's vector-memory
instruction mix and wait immediates; the library also refuses the kernel at run time if it has scratch
(ntt_plans.hpp col_db_usable).  Needs only the built library and ROCm's llvm tools (no GPU).
"""
import collections
import functools
import os
import re
import subprocess
import tempfile
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "matrix-fhe-gpu_amd" / os.environ.get("MFHE_ISA_LIB", "libmfhe.so")
LLVM = Path("/opt/rocm/lib/llvm/bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


@functools.lru_cache(maxsize=1)
def _disassembly() -> tuple:
    """llvm-objdump of every gfx950 code object in libmfhe.so (one offload bundle per translation unit)."""
    if not LIB.exists() or not (LLVM / "llvm-objdump").exists():
        pytest.skip("libmfhe.so or ROCm llvm tools missing")
    out = []
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        fb = td / "fb.bin"
        subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", str(LIB)], check=True,
                       capture_output=True)
        data = fb.read_bytes()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        for k in range(len(starts) - 1):   # one offload bundle per translation unit, concatenated
            part, co = td / f"b{k}.bin", td / f"b{k}.co"
            part.write_bytes(data[starts[k]:starts[k + 1]])
            r = subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode or not co.exists() or co.stat().st_size == 0:
                continue
            out.append(subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], capture_output=True,
                                      text=True).stdout)
    return tuple(out)


def _kernel_asm(symbol_re: str) -> str:
    for dis in _disassembly():
        m = re.search(r"^[0-9a-f]+ <(" + symbol_re + r")>:\n(.*?)(?:\n\n|\Z)", dis, re.S | re.M)
        if m:
            return m.group(2)
    pytest.fail(f"kernel {symbol_re} not found in {LIB}")


@pytest.mark.parametrize("arith,inv", [("F64", False), ("F64", True), ("U64", False), ("U64", True), ("U60", False),
                                       ("U60", True)],
                         ids=["F64-forward-first-pass", "F64-inverse-last-pass", "U64-forward-first-pass",
                              "U64-inverse-last-pass", "U60-forward-first-pass", "U60-inverse-last-pass"])
def test_column_pass_dma_waits_match_the_instruction_mix(inv, arith):
    sb = arith != "F64"   # the U64 / U60 column pass runs the single-buffer form (ntt_plans.hpp col_db_single)
    asm = _kernel_asm(r"_ZN4mfhe17ntt_col_db_kernelINS_8Arith" + arith + r"ENS_6TwSrc" + arith[0] +
                      r"ELb" + ("1" if inv else "0") + r"ELb" + ("1" if sb else "0") + r"E[^>]*")
    ops = collections.Counter(re.findall(r"^\s+((?:global|buffer|flat|scratch)_[a-z0-9_]+)", asm, re.M))
    waits = sorted({int(v) for v in re.findall(r"s_waitcnt[^\n]*vmcnt\((\d+)\)", asm)})
    # ColDb: kDmaOps = 8 DMA instructions per tile (prologue + loop body), R = 16 stores per tile: the forward's
    # intermediate (plain global stores), the inverse's output (sc1 nt buffer stores)
    store = "buffer_store_dwordx2" if inv else "global_store_dwordx2"
    # U64: + 1 DMA instruction per wave for the limb's twiddle table (issued before the limb's vmcnt(0))
    assert ops["global_load_lds_dwordx4"] == (17 if sb else 16), ops
    assert ops[store] == 16, ops
    assert not any(k.startswith("scratch_") for k in ops), ops            # no spills
    assert not any("store" in k for k in ops if k != store), ops
    # everything else is the once-per-limb twiddle / constant fetch, followed by vmcnt(0)
    other = {k: v for k, v in ops.items() if k not in ("global_load_lds_dwordx4", store)}
    assert set(other) <= {"global_load_dwordx4", "global_load_dwordx2", "global_load_dword"}, ops
    assert sum(other.values()) <= 24, ops
    if sb:
        # single buffer: the next tile's DMA is issued mid-tile, before the R = 16 stores: "tile t landed" is
        # vmcnt(16) (vmcnt(0) for the first tile and at a limb change)
        assert set(waits) <= {0, 16} and 16 in waits, waits
    else:
        # the counted waits: 8 (first tile behind the next DMA), 16 (last tile behind the stores), 24 (both)
        assert set(waits) <= {0, 8, 16, 24}, waits
        assert {8, 16, 24} <= set(waits), waits
    # and no compiler wait inside the butterflies: the tile's butterflies are one straight-line block ending in
    # its first store (the compiler lays the blocks out in varying order, so walk back from that store to the
    # previous branch or counted wait); no other vmcnt wait may sit in it (one would wait for the prefetch too)
    lines = asm.split("\n")
    s0 = next(i for i, l in enumerate(lines) if re.search(r"\b(global|buffer)_store", l))
    b0 = max(i for i in range(s0) if re.search(r"\bs_(c?branch|endpgm)|vmcnt\((8|16|24)\)", lines[i]))
    assert s0 - b0 > 300, (b0, s0)   # the block really holds the butterflies
    assert not any("vmcnt" in l for l in lines[b0 + 1:s0]), [l for l in lines[b0 + 1:s0] if "vmcnt" in l]
    # the stores' base is uniform: no readfirstlane (waterfall) loop around them
    assert "s_cbranch_execnz" not in "\n".join(lines[s0:s0 + 80]), "stores wrapped in a waterfall loop"


@pytest.mark.parametrize("kernel", [
    r"_ZN4mfhe25mfma_digitize_fold_kernelILi5ELi0E[^>]*",
    r"_ZN4mfhe25mfma_digitize_fold_kernelILi5ELi1E[^>]*",
    r"_ZN4mfhe25mfma_digitize_fold_kernelILi5ELi3E[^>]*",
    r"_ZN4mfhe26mfma_digitize_ifold_kernelILi5E[^>]*",
    r"_ZN4mfhe30mfma_digitize_ifold_dec_kernelILi6E[^>]*",
])
def test_digitize_loads_are_not_serialised(kernel):
    """The W-CRT digitize kernels (gemm.hip) must keep their column loads in flight together: a load under a
    `live ? x : 0` branch compiled to one branch per load, each followed by its own `s_waitcnt vmcnt(0)`, and a
    thread's 32 loads ran one at a time (70 -> 45 us once fixed).  Pinned here: no global load
    is followed by a vmcnt(0) within the next four instructions.  (The uniform-sampler source, SRC 2, computes its
    values and loads nothing.)"""
    asm = _kernel_asm(kernel)
    lines = [ln for ln in asm.splitlines() if re.match(r"^\s+[0-9a-f]+:", ln) or ln.startswith("\t")]
    serial = 0
    loads = 0
    for i, ln in enumerate(lines):
        if "global_load_dword" in ln:
            loads += 1
            if any("s_waitcnt vmcnt(0)" in x for x in lines[i + 1:i + 5]):
                serial += 1
    assert loads >= 2, (loads, kernel)
    assert serial <= 2, f"{serial} of {loads} loads waited for at once in {kernel}"


@pytest.mark.parametrize("D,mode", [(5, 1), (6, 1), (5, 2), (6, 2)])
def test_wcrt_ring_gemm_counted_waits(D, mode):
    """mod_gemm_mfma_ring_kernel<D, MODE, false> (gemm.hip), the default factored forward (MODE 1) and inverse
    (MODE 2) W-CRT GEMM: its K loop waits for stage s with a counted `s_waitcnt vmcnt(D)` / `vmcnt(2D)` (D = 5, four
    ring slots) or `vmcnt(D)` (D = 6, three slots) that leaves the next stages' D DMA instructions each in flight
    (ADVICE r03).  Pinned: D DMAs per 32-k stage (K = 256: 8
    stages, fully unrolled), no scratch traffic, no store and at most one other vector load between the first DMA
    and the last barrier of the K loop (an extra op issued there can only make a counted wait stricter), and only
    the immediates 0, D and 2D there.  The library also refuses a spilling ring kernel at run time (ring_usable)."""
    asm = _kernel_asm(r"_ZN4mfhe25mod_gemm_mfma_ring_kernelILi%dELi%dELb0E[^>]*" % (D, mode))
    lines = asm.split("\n")
    ops = collections.Counter(re.findall(r"^\s+((?:global|buffer|flat|scratch)_[a-z0-9_]+)", asm, re.M))
    assert not any(k.startswith("scratch_") for k in ops), ops
    dma = [i for i, ln in enumerate(lines) if "global_load_lds_dwordx4" in ln]
    assert len(dma) == 8 * D, (len(dma), D)
    bar = [i for i, ln in enumerate(lines) if "s_barrier" in ln]
    region = lines[dma[0]:bar[-1] + 1]
    other = [ln for ln in region if re.search(r"\b(global|buffer|flat)_", ln) and "global_load_lds" not in ln]
    assert not any("store" in ln or "atomic" in ln for ln in other), other
    assert len(other) <= 1, other
    waits = {int(v) for ln in region for v in re.findall(r"vmcnt\((\d+)\)", ln)}
    # ring_slots: 4 slots (stages s + 1 .. s + 3 in flight) at D = 5, 3 slots (s + 1, s + 2) at D = 6
    want = {0, D, 2 * D} if D <= 5 else {0, D}
    assert waits <= want and want - {0} <= waits, waits
    assert len(bar) == 8, len(bar)   # one barrier per stage: the prologue's and seven in the loop


@pytest.mark.parametrize("mode", [1, 2])
def test_wcrt_ring56_gemm_counted_waits(mode):
    """mod_gemm_mfma_ring56_kernel<MODE> (gemm.hip, r04): the factored launch's D = 5 and D = 6 limbs in one grid, the
    two ring bodies behind a workgroup-uniform branch.  Each body keeps its own counted waits (D = 5: vmcnt 0 / 5 / 10,
    D = 6: 0 / 6), so the kernel holds 8 x (5 + 6) DMAs, 16 barriers, no scratch, no store and at most one other
    vector load per body inside the K loops, and 2 workgroups per CU worth of registers (<= 256 VGPRs)."""
    asm = _kernel_asm(r"_ZN4mfhe27mod_gemm_mfma_ring56_kernelILi%dEEEvNS_11ModGemmArgsEjim" % mode)
    lines = asm.split("\n")
    ops = collections.Counter(re.findall(r"^\s+((?:global|buffer|flat|scratch)_[a-z0-9_]+)", asm, re.M))
    assert not any(k.startswith("scratch_") for k in ops), ops
    bar = [i for i, ln in enumerate(lines) if "s_barrier" in ln]
    assert len(bar) == 16, len(bar)
    # the two bodies are laid out one after the other: each holds 8 barriers (prologue + 7 in its K loop)
    seen = set()
    for seg in (lines[:bar[7] + 1], lines[bar[7] + 1:]):
        dma = [i for i, ln in enumerate(seg) if "global_load_lds_dwordx4" in ln]
        D = len(dma) // 8
        assert len(dma) == 8 * D and D in (5, 6), len(dma)
        seen.add(D)
        sbar = [i for i, ln in enumerate(seg) if "s_barrier" in ln]
        region = seg[dma[0]:sbar[-1] + 1]
        waits = {int(v) for ln in region for v in re.findall(r"vmcnt\((\d+)\)", ln)}
        want = {0, D, 2 * D} if D == 5 else {0, D}
        assert waits <= want and want - {0} <= waits, (D, waits)
        other = [ln for ln in region if re.search(r"\b(global|buffer|flat)_", ln) and "global_load_lds" not in ln]
        assert not any("store" in ln or "atomic" in ln for ln in other), other
        assert len(other) <= 1, other
    assert seen == {5, 6}, seen


def test_wcrt_ring_gemm_no_one_ahead_instantiation_at_d6():
    """pipe 3 (one-ahead A fragment) runs at D <= 5 only: its D = 6 form spills."""
    for mode in (0, 1, 2):
        with pytest.raises(BaseException):
            _kernel_asm(r"_ZN4mfhe25mod_gemm_mfma_ring_kernelILi6ELi%dELb1E[^>]*" % mode)


@pytest.mark.parametrize("inv", [0, 1], ids=["forward", "inverse"])
def test_single_pass_14_has_no_memory_traffic_inside_the_transform(inv):
    """ntt14_kernel (ntt_single14.hpp): the next polynomial's 16 loads per thread are issued before the transform
    and must stay in flight through it, so between the loop's prefetch and its 16 stores there is no vector-memory
    instruction (the twiddles come from LDS) and no scratch anywhere (the LICM-hoisted addresses once spilled 102
    VGPRs).  Barriers are LDS-only: no `__syncthreads()` release fence (vmcnt(0)) between the loads and the stores,
    and one per polynomial (the wave-local exchanges L1 <-> L2 <-> L3 have none, the first write waits on a counter)."""
    asm = _kernel_asm(r"_ZN4mfhe12ntt14_kernelILb%dEEEvNS_8PassArgsINS_6TwSrcFEEE" % inv)
    lines = [ln.split("//")[0].strip() for ln in asm.split("\n") if ln.strip()]
    ops = collections.Counter(re.findall(r"^\s+((?:global|buffer|flat|scratch)_[a-z0-9_]+)", asm, re.M))
    assert not any(k.startswith("scratch_") for k in ops), ops
    assert ops["buffer_load_dwordx2"] == 32 and ops["buffer_store_dwordx2"] == 16, ops
    loads = [i for i, ln in enumerate(lines) if ln.startswith("buffer_load_dwordx2")]
    stores = [i for i, ln in enumerate(lines) if ln.startswith("buffer_store_dwordx2")]
    pf_end = loads[-1]   # the in-loop prefetch is the second group of 16 loads
    # the transform runs from the prefetch to the first store in execution order: straight down when the stores
    # follow the prefetch in the code, else down to the loop's back-edge (a rotated loop keeps its stores first)
    body = lines[pf_end + 1:stores[0]] if stores[0] > pf_end else lines[pf_end + 1:]
    assert not any(re.match(r"(global|buffer|flat|scratch)_", ln) for ln in body), "vector memory inside the transform"
    # r04: one workgroup barrier per polynomial, after the cross-wave L0 image is written; the polynomial's first LDS
    # write waits on an LDS drain counter (ds_add_u32 / ds_read_b32 in inline asm), the wave-local exchanges wait for
    # their own LDS writes only (lgkmcnt)
    bars = [i for i, ln in enumerate(body) if ln.startswith("s_barrier")]
    assert len(bars) == 1, bars
    assert sum(ln.startswith("ds_add_u32") for ln in body) == 1
    # no vmcnt wait inside the transform: it would wait for the prefetch
    waits = [ln for ln in body if "vmcnt" in ln]
    assert not waits, waits[:3]
