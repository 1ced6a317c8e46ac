"""GPU, several devices: every multi-device branch of the band, run the moment
more than one GPU is visible, each checked bit for bit
against the oracle on integer data:

- one RCCL (torch "nccl") rank per GPU: ``band_reduce_dist`` (the reduce, a
  gather to the root and its stitch), ``BandPipeline`` (torch.distributed
  gather) and ``NativeBandPipeline`` (the C ABI's ncclGather on a stream of
  its own), as bench.py's N > 1 steps run them;
- one process driving several GPUs: ``bldp_band_reduce_multi_f32`` on its
  default branch (the root's launch stores its slots, every other device one
  launch into staging + one peer copy), its staged branch, and the opt-in
  direct xGMI store branch (``BLDP_BAND_PEER_STORE``), for contiguous and
  round-robin bank placements;
- ``GBT.getband`` with its banks' workers on several GPUs (raw band read and
  bank-by-bank decode);
- ``bench.py --gpus N`` itself, which checks its own stitched band.

The reference fans one worker out per bank and stitches with
``reduce(vcat, fetch.(futures))`` (src/gbt.jl:75-78,103).  On a one-GPU box
every test here skips with the reason; the single-device forms of the same
code run in test_gpu_parity.py / test_gpu_api.py."""
from __future__ import annotations

import os

import numpy as np
import pytest

from conftest import REPO, same_bits

pytestmark = pytest.mark.gpu


def _ndev() -> int:
    import torch

    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def _world() -> int:
    """Ranks for the 8-bank band: the most of 8, 4, 2 GPUs visible."""
    n = _ndev()
    return next((w for w in (8, 4, 2) if w <= n), 1)


def _need_gpus(n=2):
    if _ndev() < n:
        pytest.skip(f"needs >= {n} GPUs, {_ndev()} visible: the multi-device branches run on a "
                    "multi-GPU node (single-device forms: test_gpu_parity.py, test_gpu_api.py)")


def _int_banks(seed, nb, shape):
    rng = np.random.default_rng(seed)
    return [np.asfortranarray(rng.integers(0, 256, shape).astype(np.float32)) for _ in range(nb)]


def _rank_main(rank, world, port, q, kind, cases):
    """One RCCL rank on GPU ``rank``: its contiguous banks, each case's exchange
    checked on the root against the oracle's stitched band (bit-exact)."""
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    import __graft_entry__ as entry

    pkg, orc = entry.load_package(), entry.load_oracle()
    eng = pkg.engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world,
                            device_id=torch.device("cuda", rank))
    ok = []
    for shape, F, T, win in cases:
        banks = _int_banks(500 + F + T, 8, shape)
        mine = list(pkg.band.banks_for_rank(8, rank, world))
        dbanks = [eng.fb_from_numpy(banks[b], f"cuda:{rank}") for b in mine]
        want = orc.stitch([orc.reduce(b, F, T, "sum", win) for b in banks])
        if kind == "dist":
            res = pkg.band.band_reduce_dist(dbanks, F, T, "sum", win)
            got = [eng.fb_to_numpy(res)] if rank == 0 else [res]
        else:
            nco, ni, nto = eng.out_shape(shape, win, F, T)
            if kind == "native":
                pipe = pkg.band.NativeBandPipeline(len(mine) * nco, ni, nto,
                                                   device=f"cuda:{rank}")
            else:
                pipe = pkg.band.BandPipeline(len(mine) * nco, ni, nto, device=f"cuda:{rank}")
            got = []
            for _ in range(3):  # slots reused: step k's gather overlaps step k+1's reduce
                s = pipe.begin()
                eng.band_reduce(dbanks, F, T, "sum", win, out=pipe.local(s))
                r = pipe.exchange(s)
                pipe.wait(s)
                torch.cuda.synchronize()
                got.append(eng.fb_to_numpy(r) if rank == 0 else r)
            pipe.drain()
            if kind == "native":
                pipe.close()
        for g in got:
            ok.append(same_bits(g, want) if rank == 0 else g is None)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, ok))


@pytest.mark.parametrize("kind", ["dist", "torch", "native"])
def test_rccl_ranks_band_exchange(kind):
    """bench.py's N > 1 exchange with one RCCL rank per GPU (2, 4 or 8 ranks):
    single-row products (the gathered bytes are the band) and many-row ones
    (the root's stitch kernel)."""
    _need_gpus(2)
    import torch.multiprocessing as mp

    world = _world()
    cases = [((8192, 1, 16), 1024, 16, None),
             ((4096, 2, 40), 64, 8, [0, 4096, 1, 0, 2, 1, 0, 32, 1])]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31000 + os.getpid() % 500 + {"dist": 0, "torch": 1, "native": 2}[kind]
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, q, kind, cases))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=240)
    for p in ps:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    res = dict(q.get(timeout=5) for _ in ps)
    assert all(res[r] and all(res[r]) for r in range(world)), res


@pytest.mark.parametrize("placement", ["contiguous", "round-robin"])
@pytest.mark.parametrize("mode", ["default", "staged", "peer_store"])
def test_band_reduce_multi_across_devices(pkg, orc, placement, mode):
    """bldp_band_reduce_multi_f32 with banks on several GPUs: contiguous
    shards (one launch per device) and round-robin ones (one launch per device
    whose banks' slots are `ndev` slots apart; staged runs copied bank by
    bank).  Bit-exact against the oracle, a one-row and a many-row product."""
    _need_gpus(2)
    import torch

    eng = pkg.engine
    n = min(_ndev(), 8)
    for shape, F, T, win in (((8192, 1, 16), 1024, 16, None),
                             ((4096, 3, 40), 16, 8, [8, 4080, 1, 0, 3, 1, 0, 40, 1])):
        banks = _int_banks(900 + F, 8, shape)
        devs = ([b * n // 8 for b in range(8)] if placement == "contiguous"
                else [b % n for b in range(8)])
        xs = [eng.fb_from_numpy(a, f"cuda:{d}") for a, d in zip(banks, devs)]
        want = orc.stitch([orc.reduce(a, F, T, "sum", win) for a in banks])
        for root in (0, n - 1):
            got = eng.band_reduce_multi(xs, F, T, "sum", win, root=root,
                                        staged=mode == "staged", peer_store=mode == "peer_store")
            assert got.device == torch.device("cuda", root)
            assert same_bits(eng.fb_to_numpy(got), want), (shape, placement, mode, root)


@pytest.mark.parametrize("peer_store", [False, True])
@pytest.mark.parametrize("branch", ["raw band", "bank by bank"])
def test_getband_banks_on_several_gpus(pkg, orc, tmp_path, monkeypatch, peer_store, branch):
    """GBT.getband with its banks' workers on several GPUs: the raw band read
    (each GPU reads its banks as one stream, one reduce per GPU into the
    root's slots) and the bank-by-bank branch (compressed banks decoded on
    their GPU; the slot filled by the root's own store, a device copy, or with
    peer_store a kernel store over xGMI).  Bit-exact against the oracle, with
    despike (src/gbt.jl:75-78,101-103)."""
    _need_gpus(2)
    n = min(_ndev(), 8)
    C = pkg.COLON
    banks = _int_banks(4711, 8, (4096, 1, 48))
    names = []
    for b, a in enumerate(banks):
        hdr = dict(foff=-187.5 / 4096, fch1=8400.0 - 187.5 * b, nfpc=64)
        f = str(tmp_path / f"m{b}.rawspec.0002.h5")
        if branch == "raw band":
            pkg.fbh5.write(f, hdr, a)
        else:
            pkg.fbh5.write_bslz4(f, hdr, a, (16, 1, 4096),
                                 lambda blk: orc.np_bslz4_encode(blk, 512, lz4=orc.lz4_compress))
        names.append(f)
    if branch == "bank by bank":
        monkeypatch.setattr(pkg.GBT, "_band_chunked", lambda *a, **k: False)
    for workers in ([b * n // 8 for b in range(8)], [(b + 1) % n for b in range(8)]):
        tm = {}
        got = pkg.GBT._band_on_device(workers, names, (C, C, C), 64, "sum", 16, 64,
                                      timings=tm, peer_store=peer_store)
        assert tm["path"] == branch, tm
        want = orc.despike(orc.stitch([orc.reduce(a, 64, 16) for a in banks]), 64)
        assert same_bits(got, want), (workers, branch, peer_store)


def test_bench_verifies_its_multi_gpu_band():
    """bench.py --gpus N (N = 2, 4 or 8; ranks started by bench.py itself, one
    RCCL rank per GPU) prints one line whose stitched band it checked bit for
    bit on integer data after the timed region ("verified": true)."""
    _need_gpus(2)
    import json
    import subprocess
    import sys

    world = _world()
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    for cfg in ("cfg2", "cfg3"):
        r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(world),
                            "--config", cfg, "--steps", "3", "--warmup", "1",
                            "--no-cpu-baseline", "--no-read-probe", "--rank-deadline", "400"],
                           capture_output=True, text=True, timeout=480, env=env)
        assert r.returncode == 0, (cfg, r.returncode, r.stderr[-3000:])
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        d = json.loads(lines[0])
        assert d["n_gpus"] == world and d["verified"] is True, d.get("verify")
