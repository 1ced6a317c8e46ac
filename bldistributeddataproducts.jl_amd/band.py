"""A band across GPUs: one process per GPU, banks sharded by rank, one
exchange step (RCCL gather over xGMI) and the band stitch on the root.

The reference fans ``WorkerFunctions.getdata`` out over one Distributed.jl
worker per bank and gathers with ``fetch.(futures)`` (src/gbt.jl:75-78); the
stitch is ``reduce(vcat, ...)`` in bank order (src/gbt.jl:103).  Here:

1. rank r owns the contiguous banks ``banks_for_rank(nbank, r, world)``;
2. it reduces them with ONE launch that already writes its slice of the band
   in stitched order (``engine.band_reduce``);
3. ``torch.distributed.gather`` (backend "nccl" = RCCL) brings every rank's
   slice to the root, which leaves rank-major blocks;
4. the root permutes rank-major -> vcat with ``bldp_stitch_f32``.  When every
   bank's output is a single (IF, time) row the gathered bytes already are the
   stitched product and step 4 is skipped.

Reduce-then-gather is exact because fqavby divides the per-bank channel count,
so no decimation group straddles two banks.
"""
from __future__ import annotations


def banks_for_rank(nbank: int, rank: int, world: int) -> range:
    """Contiguous block of banks owned by ``rank`` (bank order == rank order)."""
    if nbank % world:
        raise ValueError(f"{nbank} banks do not shard evenly over {world} ranks")
    per = nbank // world
    return range(rank * per, (rank + 1) * per)


def band_reduce_dist(local_banks, fqavby=1, tavby=1, op="sum", win=None, root=0, group=None,
                     reduce_fn=None, stitch_fn=None, out=None):
    """SPMD: every rank passes its own banks; the root returns the stitched
    (nbank*nco, ni, nto) product, other ranks return None.

    ``reduce_fn(banks, fqavby, tavby, op, win) -> (nbl*nco, ni, nto)`` and
    ``stitch_fn(gathered[world, nto, ni, nbl*nco], world) -> product`` default
    to the HIP engine; tests inject CPU stand-ins to exercise the sharding and
    exchange logic under the gloo backend."""
    import torch
    import torch.distributed as dist

    from . import engine

    reduce_fn = reduce_fn or (lambda b, F, T, o, w: engine.band_reduce(b, F, T, o, w))
    stitch_fn = stitch_fn or (lambda g, n: engine.stitch(g, n))
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    local = reduce_fn(list(local_banks), fqavby, tavby, op, win)  # (nbl*nco, ni, nto)
    ncl, ni, nto = local.shape
    # contiguous [nto][ni][ncl] bytes of this rank's slice
    block = local.permute(2, 1, 0).contiguous() if local.dim() == 3 else local
    if world == 1:
        return local
    dev = block.device
    if dist.get_backend(group) == "gloo" and block.is_cuda:
        block = block.cpu()  # gloo rehearsal of the N-rank path (CPU transport)
    if rank == root:
        gathered = torch.empty((world, nto, ni, ncl), dtype=block.dtype, device=block.device)
        dist.gather(block, gather_list=list(gathered.unbind(0)), dst=root, group=group)
        gathered = gathered.to(dev)
        if ni * nto == 1:
            res = gathered.reshape(world * ncl, 1, 1)
            if out is not None:
                out.copy_(res)
                return out
            return res
        return stitch_fn(gathered, world)
    dist.gather(block, gather_list=None, dst=root, group=group)
    return None
