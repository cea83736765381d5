"""Multi-GPU residue sharding: RCCL exchange + in-place sharded CRT recombine.

Layout: with `world` ranks and L limbs, rank g owns limbs [g*Lg, (g+1)*Lg), Lg = L / world, for every
polynomial of the batch: a [batch][Lg][ncoeff] u64 shard (NTT, RNS decompose and W-CRT are
per-limb and need no communication).  Wide CRT recombine needs all L residues of a coefficient,
so it is the one exchange step.  Rank g recombines the batch slice [g*B/world, (g+1)*B/world):

  allgather : all_gather_into_tensor -> [world][batch][Lg][n]; every rank receives (world-1)/world
              of the whole residue set and composes its slice in place.
  alltoall  : all_to_all_single       -> [world][batch/world][Lg][n]; every rank receives only the
              missing limbs of its own slice ((world-1)/world^2 of the residue set).

Both hand the received buffer to mfhe_crt_compose_f64_sharded, which reads the shards in place
(no transpose).  On GPU the whole step is one C-ABI call, mfhe_crt_recombine_sharded, over an RCCL
communicator owned by libmfhe (mfhe.Comm; receive buffer preallocated by crt_recombine_reserve), so a C++
caller of the reference API shards residues the same way.  exchange_residues restates the exchange with
torch.distributed collectives: it is what the gloo CPU tests drive to pin the shard layout the native
call produces (same offsets, same strides).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def limb_range(L: int, world: int, rank: int) -> tuple[int, int]:
    """(start_limb, nlimbs) owned by `rank` under residue sharding."""
    if L % world:
        raise ValueError(f"L={L} must be a multiple of world={world}")
    lg = L // world
    return rank * lg, lg


def exchange_residues(shard: torch.Tensor, batch: int, lg: int, ncoeff: int, mode: str = "allgather", group=None):
    """Exchange this rank's [batch][lg][ncoeff] residue shard.

    Returns (buf, offset, shard_stride, npoly): this rank's batch slice is `world` shards starting at
    word `offset` of `buf`, `shard_stride` words apart, each [npoly][lg][ncoeff].
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if shard.numel() != batch * lg * ncoeff:
        raise ValueError("shard size does not match batch * lg * ncoeff")
    if batch % world:
        raise ValueError(f"batch={batch} must be a multiple of world={world}")
    bs = batch // world
    shard = shard.reshape(-1)
    if mode == "allgather":
        buf = torch.empty(world * shard.numel(), dtype=shard.dtype, device=shard.device)
        dist.all_gather_into_tensor(buf, shard, group=group)
        return buf, rank * bs * lg * ncoeff, batch * lg * ncoeff, bs
    if mode == "alltoall":
        buf = torch.empty(world * bs * lg * ncoeff, dtype=shard.dtype, device=shard.device)
        dist.all_to_all_single(buf, shard, group=group)   # chunk r of the input = polys of rank r's slice
        return buf, 0, bs * lg * ncoeff, bs
    raise ValueError(f"unknown exchange mode {mode!r}")


def chunk_plan(batch: int, world: int, chunk_polys: int) -> list[tuple[int, int, int]]:
    """Recombine in poly chunks to bound the receive buffer (BASELINE C5: the whole all-gather would be
    112 GiB per GPU).  Returns [(p0, cp, row0)]: polys [p0, p0 + cp) are exchanged together (cp a multiple of
    `world`) and this rank's cp / world composed polys land at output rows [row0, row0 + cp / world)."""
    if batch % world:
        raise ValueError(f"batch={batch} must be a multiple of world={world}")
    cp = max(world, chunk_polys // world * world)
    plan, p0 = [], 0
    while p0 < batch:
        c = min(cp, batch - p0)
        plan.append((p0, c, p0 // world))
        p0 += c
    return plan


def owned_polys(batch: int, world: int, rank: int, chunk_polys: int) -> list[int]:
    """Global poly index of each output row of `rank` under chunk_plan (row order)."""
    out = []
    for p0, cp, _ in chunk_plan(batch, world, chunk_polys):
        bs = cp // world
        out += list(range(p0 + rank * bs, p0 + (rank + 1) * bs))
    return out


def crt_recombine_chunked(ctx, shard: torch.Tensor, batch: int, ncoeff: int, mode: str, chunk_polys: int,
                          out: torch.Tensor, group=None, stream=None, comm=None, rows_global: bool = False,
                          flags: int = 0) -> torch.Tensor:
    """crt_recombine over chunk_plan's poly chunks: shard [batch][Lg][ncoeff] -> out f64, rows in owned_polys
    order ([batch/world][ncoeff]) or, with rows_global, at the global poly index ([batch][ncoeff], only this
    rank's rows written).  Each chunk is one exchange + in-place sharded compose.  With `comm` the whole loop is
    the native pipelined call (mfhe_crt_recombine_chunked: chunk k + 1's RCCL exchange on the communicator's
    stream beside chunk k's compose); without it, the torch.distributed restatement below, chunk after chunk,
    which the gloo tests use to pin the same row order."""
    if comm is not None:
        return ctx.crt_recombine_chunked(comm, mode, shard, batch, ncoeff, chunk_polys, out, stream=stream,
                                         rows_global=rows_global, flags=flags)
    if flags:
        raise ValueError("crt_recombine_chunked: flags need the native path (comm)")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lg = ctx.info().num_limbs // world
    for p0, cp, row0 in chunk_plan(batch, world, chunk_polys):
        sh = shard[p0 * lg * ncoeff:(p0 + cp) * lg * ncoeff]
        r = p0 + rank * (cp // world) if rows_global else row0
        o = out[r * ncoeff:(r + cp // world) * ncoeff]
        crt_recombine(ctx, sh, cp, ncoeff, mode, group, out=o, stream=stream, comm=comm)
    return out


def decode_recombine(ctx, shard: torch.Tensor, lanes: int, ncoeff: int, mode: str, chunk_polys: int,
                     out: torch.Tensor, group=None) -> torch.Tensor:
    """The recombine step of mfhe_decode_sharded (he.hip decode_sharded_impl), restated over torch.distributed:
    the chunked recombine with rows at their lane index, then one in-place all-gather per chunk, after which
    every rank holds all `lanes` rows [lanes][ncoeff] in lane order (chunk k's lanes are [rank][cp / G])."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    crt_recombine_chunked(ctx, shard, lanes, ncoeff, mode, chunk_polys, out, group=group, rows_global=True)
    for p0, cp, _ in chunk_plan(lanes, world, chunk_polys):
        bs = cp // world
        parts = list(out[p0 * ncoeff:(p0 + cp) * ncoeff].view(world, bs * ncoeff).unbind(0))
        mine = parts[rank].clone()
        dist.all_gather(parts, mine, group=group)
    return out


def crt_recombine(ctx, shard: torch.Tensor, batch: int, ncoeff: int, mode: str = "allgather", group=None,
                  out: torch.Tensor | None = None, stream=None, comm=None) -> torch.Tensor:
    """Exchange residue shards and compose this rank's batch slice to f64 (centred value / delta).

    `ctx` is an mfhe.Context over all L moduli (its CRT tables); returns [batch/world][ncoeff] f64.
    With `comm` (an mfhe.Comm) the exchange + compose is the native mfhe_crt_recombine_sharded (RCCL);
    without it the exchange goes through torch.distributed on `group`.
    """
    if comm is not None:
        if out is None:
            out = torch.empty(batch // comm.size * ncoeff, dtype=torch.float64, device=shard.device)
        return ctx.crt_recombine_sharded(comm, mode, shard, batch, ncoeff, out, stream=stream)
    world = dist.get_world_size(group)
    L = ctx.info().num_limbs
    _, lg = limb_range(L, world, 0)
    buf, off, stride, bs = exchange_residues(shard, batch, lg, ncoeff, mode, group)
    if out is None:
        out = torch.empty(bs * ncoeff, dtype=torch.float64, device=shard.device)
    ctx.crt_compose_f64_sharded(buf, out, world, stride, bs, ncoeff, stream=stream, src_offset=off)
    return out
