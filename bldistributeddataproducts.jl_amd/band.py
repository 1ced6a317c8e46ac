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


class BandPipeline:
    """Repeated band exchange with the gather of step k overlapping the
    reduce of step k+1 (``depth`` buffer slots, asynchronous gathers).

    Per step, SPMD on every rank::

        s = pipe.begin()                     # a free slot (GPU-side wait only)
        engine.band_reduce(my_banks, ..., out=pipe.local(s))
        product = pipe.exchange(s)           # root: the stitched band; else None

    ``local(s)`` is this rank's (nbl*nco, ni, nto) Julia-order slice.  The
    gather runs on the process group's own stream; the root's product of slot
    ``s`` may still be in flight: ``wait(s)`` (or ``drain()``) makes the
    current stream wait for it.  It stays valid until that slot is used again
    ``depth`` steps later (when
    every bank's output is one (IF, time) row the gathered bytes already are
    the product, otherwise the root stitches after waiting for the gather).
    ``drain()`` waits for every gather in flight.  With the gloo backend (CPU
    transport, the rehearsal of the N-rank path) every gather completes inside
    ``exchange``.
    """

    def __init__(self, ncl, ni, nto, device, depth=2, root=0, group=None, stitch_fn=None,
                 gather_single=False):
        import torch
        import torch.distributed as dist

        from . import engine

        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.root, self.group, self.depth = root, group, depth
        self.gather_single = gather_single  # one rank: gather + stitch anyway (tests)
        self.shape = (ncl, ni, nto)
        self.gloo = dist.get_backend(group) == "gloo"
        self.stitch_fn = stitch_fn or (lambda g, n: engine.stitch(g, n))
        dev = torch.device(device)
        # Julia order (ncl, ni, nto), channel fastest = contiguous [nto][ni][ncl]
        self._local = [torch.empty((nto, ni, ncl), dtype=torch.float32, device=dev)
                       for _ in range(depth)]
        self._gathered = None
        if self.rank == root:
            gdev = torch.device("cpu") if self.gloo else dev
            self._gathered = [torch.empty((self.world, nto, ni, ncl), dtype=torch.float32,
                                          device=gdev) for _ in range(depth)]
        self._work = [None] * depth
        self._next = 0

    def local(self, slot):
        return self._local[slot].permute(2, 1, 0)

    def begin(self):
        """Next slot; the current stream waits (on the GPU) for the gather
        that last read it."""
        s = self._next
        self._next = (s + 1) % self.depth
        w = self._work[s]
        if w is not None:
            w.wait()
            self._work[s] = None
        return s

    def exchange(self, slot):
        import torch.distributed as dist

        block = self._local[slot]
        if self.world == 1 and not self.gather_single:
            return self.local(slot)
        if self.gloo and block.is_cuda:
            block = block.cpu()
        glist = list(self._gathered[slot].unbind(0)) if self.rank == self.root else None
        w = dist.gather(block, gather_list=glist, dst=self.root, group=self.group,
                        async_op=True)
        ncl, ni, nto = self.shape
        if self.gloo:
            w.wait()
        else:
            self._work[slot] = w
        if self.rank != self.root:
            return None
        g = self._gathered[slot]
        if self.gloo:
            g = g.to(self._local[slot].device)
        if ni * nto == 1:  # rank-major slices of single rows are already vcat order
            return g.reshape(self.world * ncl, 1, 1)
        if self._work[slot] is not None:
            self._work[slot].wait()  # the stitch reads the gathered blocks
            self._work[slot] = None
        return self.stitch_fn(g, self.world)

    def wait(self, slot):
        w = self._work[slot]
        if w is not None:
            w.wait()
            self._work[slot] = None

    def drain(self):
        for s, w in enumerate(self._work):
            if w is not None:
                w.wait()
                self._work[s] = None


class NativeBand:
    """The band exchange through the C ABI alone (bldp_comm_* +
    bldp_band_gather_f32: RCCL ncclGather over xGMI), the path a host without
    torch -- a Julia Distributed.jl worker per GPU -- takes.  ``id_bytes``
    (128) comes from ``NativeBand.new_id()`` on one rank and is passed to every
    rank by the host's own means.  Construction is collective."""

    def __init__(self, device, nranks, rank, id_bytes):
        import ctypes

        from . import _lib

        self.L = _lib.lib()
        self.nranks, self.rank = int(nranks), int(rank)
        self.device = int(device)
        idb = (ctypes.c_uint8 * _lib.BLDP_COMM_ID_BYTES).from_buffer_copy(bytes(id_bytes))
        h = ctypes.c_void_p()
        _lib.check(self.L.bldp_comm_init(self.device, self.nranks, self.rank, idb,
                                         ctypes.byref(h)), "bldp_comm_init")
        self.handle = h

    @staticmethod
    def new_id() -> bytes:
        import ctypes

        from . import _lib

        buf = (ctypes.c_uint8 * _lib.BLDP_COMM_ID_BYTES)()
        _lib.check(_lib.lib().bldp_comm_id(buf), "bldp_comm_id")
        return bytes(buf)

    def gather_into(self, block, gathered, root=0, stream=None):
        """Raw exchange: the dense ``block`` (every rank the same size) lands
        rank-major in ``gathered`` (root only; None elsewhere), queued on
        ``stream``."""
        from . import _lib

        if not block.is_contiguous() or (gathered is not None and not gathered.is_contiguous()):
            raise ValueError("gather_into: dense blocks only")
        if gathered is not None and gathered.numel() != self.nranks * block.numel():
            raise ValueError("gather_into: gathered holds %d floats, not %d x %d"
                             % (gathered.numel(), self.nranks, block.numel()))
        _lib.check(self.L.bldp_band_gather_f32(self.handle, int(root), block.data_ptr(),
                                               block.numel(), gathered.data_ptr()
                                               if gathered is not None else None,
                                               _lib.stream_ptr(stream)),
                   "bldp_band_gather_f32")

    def gather(self, local, root=0, stream=None):
        """``local``: this rank's Julia-order (ncl, ni, nto) slice, dense.
        Returns the stitched band on the root (a new tensor), None elsewhere."""
        import torch

        from . import _lib, engine

        ncl, ni, nto = (int(x) for x in local.shape)
        block = local.permute(2, 1, 0)
        if not block.is_contiguous():
            raise ValueError("local slice must be a dense Julia-order tensor")
        g = None
        if self.rank == root:
            g = torch.empty((self.nranks, nto, ni, ncl), dtype=torch.float32,
                            device=local.device)
        _lib.check(self.L.bldp_band_gather_f32(self.handle, int(root), block.data_ptr(),
                                               ncl * ni * nto, g.data_ptr() if g is not None
                                               else None, _lib.stream_ptr(stream)),
                   "bldp_band_gather_f32")
        if g is None:
            return None
        if ni * nto == 1:
            return g.reshape(self.nranks * ncl, 1, 1)
        return engine.stitch(g, self.nranks, stream=stream)

    def close(self):
        if self.handle:
            from . import _lib

            _lib.check(self.L.bldp_comm_destroy(self.handle), "bldp_comm_destroy")
            self.handle = None


class NativeBandPipeline:
    """``BandPipeline``'s interface over the C-ABI exchange: every step's
    gather is ``bldp_band_gather_f32`` (RCCL ncclGather) queued on a stream of
    the pipeline's own, after an event on the reducing stream, so it runs on
    another hardware queue beside the next step's reduce.  On MI355X this costs
    the step ~10 us against ~27 us for torch.distributed.gather, whose
    work lands on the reducing stream's queue (``tools/stream_probe.py``,
    ``profiles/r02/stream_probe.json``).

    The communicator is made from the process group: the root draws the
    RCCL id and ``broadcast_object_list`` hands it to every rank (pass
    ``comm=`` to reuse a ``NativeBand``)."""

    def __init__(self, ncl, ni, nto, device, depth=2, root=0, group=None, stitch_fn=None,
                 comm=None, priority=-1):
        import torch
        import torch.distributed as dist

        from . import engine

        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.root, self.depth = root, depth
        self.shape = (ncl, ni, nto)
        self.stitch_fn = stitch_fn or (lambda g, n: engine.stitch(g, n))
        dev = torch.device(device)
        self._own = comm is None
        if comm is None:
            obj = [NativeBand.new_id() if self.rank == root else None]
            dist.broadcast_object_list(obj, src=root, group=group)
            comm = NativeBand(dev.index if dev.index is not None else torch.cuda.current_device(),
                              self.world, self.rank, obj[0])
        self.comm = comm
        self._local = [torch.empty((nto, ni, ncl), dtype=torch.float32, device=dev)
                       for _ in range(depth)]
        self._gathered = [torch.empty((self.world, nto, ni, ncl), dtype=torch.float32,
                                      device=dev) for _ in range(depth)] \
            if self.rank == root else [None] * depth
        # high priority: HIP gives it a hardware queue of its own, so the
        # gather never sits behind the next reduce (a normal-priority stream
        # may share the reducing stream's queue, GPU_MAX_HW_QUEUES = 4)
        self.stream = torch.cuda.Stream(device=dev, priority=priority)
        self._reduced = [torch.cuda.Event() for _ in range(depth)]
        self._done = [torch.cuda.Event() for _ in range(depth)]
        self._pending = [False] * depth
        self._next = 0

    def local(self, slot):
        return self._local[slot].permute(2, 1, 0)

    def begin(self):
        """Next slot; the current stream waits (on the GPU) for the gather
        that last read it."""
        s = self._next
        self._next = (s + 1) % self.depth
        self.wait(s)
        return s

    def exchange(self, slot):
        import torch

        cur = torch.cuda.current_stream()
        self._reduced[slot].record(cur)
        self.stream.wait_event(self._reduced[slot])
        self.comm.gather_into(self._local[slot], self._gathered[slot], self.root, self.stream)
        self._done[slot].record(self.stream)
        self._pending[slot] = True
        if self.rank != self.root:
            return None
        ncl, ni, nto = self.shape
        g = self._gathered[slot]
        if ni * nto == 1:  # rank-major slices of single rows are already vcat order
            return g.reshape(self.world * ncl, 1, 1)
        self.wait(slot)  # the stitch reads the gathered blocks
        return self.stitch_fn(g, self.world)

    def wait(self, slot):
        import torch

        if self._pending[slot]:
            torch.cuda.current_stream().wait_event(self._done[slot])
            self._pending[slot] = False

    def drain(self):
        for s in range(self.depth):
            self.wait(s)

    def close(self):
        if self._own and self.comm is not None:
            import torch

            self.stream.synchronize()
            torch.cuda.current_stream().synchronize()
            self.comm.close()
        self.comm = None
