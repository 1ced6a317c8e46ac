#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on MI355X:
"filterbank GB/s reduced (node) + % HBM roofline, 8-bank 0000 band".

Default workload (configs[2], the north-star band): 8 banks of 0000-product
data, each (2^26 channels x 1 IF x 16 spectra) Float32 = 4 GiB, frequency
decimated by 1024 and time integrated by 16, stitched into one
(524288, 1, 1) band product.  The band is one fixed job (strong scaling):
with N GPUs each rank owns 8/N contiguous banks (one launch reduces them all
into its stitched slice), RCCL gathers the slices to rank 0 over xGMI and rank
0 stitches.  At N=1 one GPU holds all 32 GiB and does the whole band in a
single launch.

A step = one pass of the hot path over the band, inputs resident in HBM.
Algorithmic bytes per step = 4*nchan*nif*ntime read + 4*(nchan/F)*nif*(ntime/T)
written, summed over banks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg3]
    torchrun --nproc-per-node N bench.py --gpus N ...   (N > 1)
    python bench.py --gpus N ...   (N > 1, no launcher: bench.py starts the N
                                    rank processes itself, see spawn_ranks)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "filterbank GB/s reduced (node) + % HBM roofline, 8-bank 0000 band"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    # BASELINE.json configs[0]: 0002 single bank (the reference's CPU case)
    "cfg1": dict(workload="0002 single bank (65536 ch x 1 IF x 279 spectra), window t=1:272, "
                 "F=64 T=16", nbank=1, nchan=65536, nif=1, ntime=279, tw=272, F=64, T=16,
                 nfpc=1024, product=2),
    # configs[1]: 8 banks of 0002 stitched on one GPU
    "cfg2": dict(workload="0002 band: 8 banks (65536 ch x 1 IF x 279), window t=1:272, F=64 "
                 "T=16, stitched to 524288 ch", nbank=8, nchan=65536, nif=1, ntime=279, tw=272,
                 F=64, T=16, nfpc=1024, product=2),
    # configs[2]: the north star
    "cfg3": dict(workload="0000 band: 8 banks x (2^26 ch x 1 IF x 16 spectra) = 32 GiB, F=1024 "
                 "T=16, stitched to 524288 ch (RCCL gather when N>1)", nbank=8, nchan=1 << 26,
                 nif=1, ntime=16, tw=16, F=1024, T=16, nfpc=1 << 20, product=0),
    # gather-stress variant of configs[2]: time integration only
    "cfg3f1": dict(workload="0000 band, F=1 T=16 (256 MiB/bank output, gather-stress)",
                   nbank=8, nchan=1 << 26, nif=1, ntime=16, tw=16, F=1, T=16, nfpc=1 << 20,
                   product=0),
    # configs[3]: 0001 high-time-resolution banks
    "cfg4": dict(workload="0001 band: 8 banks (512 ch x 1 IF x 880000 spectra), window "
                 "t=1:879616, F=8 T=1024", nbank=8, nchan=512, nif=1, ntime=880000, tw=879616,
                 F=8, T=1024, nfpc=8, product=1),
}


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


COLD_BYTES = 1 << 30  # > 4x the 256 MB Infinity Cache (MI355X_MICROARCH.md)


def cold_copies(mode, launch_bytes):
    """Distinct copies of a launch's input the steps rotate over: 1 (warm, or
    a launch too big for any cache), else enough for >= COLD_BYTES."""
    if mode == "warm" or (mode == "auto" and launch_bytes >= COLD_BYTES) or launch_bytes <= 0:
        return 1
    return max(2, min(64, -(-COLD_BYTES // launch_bytes)))


def cache_note(ncopy, launch_bytes):
    if ncopy == 1:
        return ("one copy: every launch re-reads the same buffer" +
                (" (larger than any cache: HBM-bound)" if launch_bytes >= COLD_BYTES else
                 " (warm: the Infinity Cache may hold part of it)"))
    return (f"cold: launches rotate over {ncopy} copies of the input "
            f"({ncopy * launch_bytes / 2**20:.0f} MiB), none in cache from the launch before")


def traffic_from_profile(cfg_name, n_local_banks, with_source=False):
    """HBM bytes per launch from the committed PMC profile (profiles/), or None.
    with_source: (bytes, where they come from) — a committed counter session,
    not a measurement taken in this run."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return (None, None) if with_source else None
    e = d.get(cfg_name, {}).get(str(n_local_banks))
    b = e.get("hbm_bytes_per_launch") if e else None
    if not with_source:
        return b
    src = None
    if e:
        files = e.get("source") or []
        src = (f"profiles/pmc_traffic.json [{cfg_name!r}][{str(n_local_banks)!r}]: committed "
               f"rocprofv3 --pmc session ({', '.join(files) or 'per-kernel medians'}; "
               f"{e.get('correction', '')}), not measured in this run")
    return b, src


def host_cpu_info():
    """The host this runs on: CPU model, the machine's logical CPUs (nproc)
    and the CPUs this process may use (the GPU box's share of a node)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return {"cpu_model": model, "host_nproc": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": int(omp) if omp.isdigit() else None}


def cpu_baseline(cfg, seconds, eng, torch):
    """The oracle (C restatement) on the FULL banks of the workload, on this
    host's cores: one pthread per bank (GBT.getdata's one Distributed worker
    per bank, src/gbt.jl:75-77) is the baseline; the same arithmetic over a
    pool of every CPU this process may use is reported beside it."""
    import __graft_entry__ as entry

    orc = entry.load_oracle()
    nb = cfg["nbank"]
    nch, nt = cfg["nchan"], cfg["tw"] - cfg["tw"] % cfg["T"]
    banks = []
    for b in range(nb):  # the window's bytes, generated on the GPU, copied to host memory
        t = eng.synth(nch, cfg["nif"], nt, cfg["nfpc"], seed=10 * b + cfg["product"], kind=0)
        banks.append(eng.fb_to_numpy(t))
        del t
    torch.cuda.empty_cache()
    per_rep = nb * 4 * (nch * cfg["nif"] * nt + (nch // cfg["F"]) * cfg["nif"] * (nt // cfg["T"]))
    info = host_cpu_info()
    # the pool runs on the box's CPU share (OMP_NUM_THREADS, 16 on the GPU
    # box), not on every CPU the host has (host_nproc) or this process could
    # be scheduled on (affinity_cpus): the key names the thread count
    nthr = info["omp_num_threads"] or info["affinity_cpus"]

    def timed(fn, secs):
        fn()  # warm (page faults)
        reps, t0 = 0, time.perf_counter()
        while True:
            fn()
            reps += 1
            el = time.perf_counter() - t0
            if el >= secs and reps >= 2:
                return per_rep * reps / el / 1e9, reps, el

    gbs, reps, el = timed(lambda: orc.reduce_banks_mt(banks, cfg["F"], cfg["T"]), 0.6 * seconds)
    gall, reps_all, el_all = timed(
        lambda: orc.reduce_banks_pool(banks, cfg["F"], cfg["T"], "sum", nthr), 0.4 * seconds)
    return dict({"value": round(gbs, 3), "unit": "GB/s", "cores": nb, "kind": "port",
                 "sample": f"the full workload: {nb} banks x ({nch} ch x {cfg['nif']} IF x {nt} "
                           f"spectra), F={cfg['F']} T={cfg['T']}, {reps} passes in {el:.1f} s; "
                           "oracle/bldp_oracle.c (Float64 accumulate, gcc -O3 x86-64-v3), "
                           "one pthread per bank as one Distributed worker per bank",
                 f"pool_{nthr}_threads": {
                     "value": round(gall, 3), "threads": nthr,
                     "sample": f"same banks, output channels split over {nthr} threads "
                               f"(OMP_NUM_THREADS, this box's CPU share; not all "
                               f"{info['host_nproc']} host CPUs), {reps_all} passes in "
                               f"{el_all:.1f} s"}},
                **info)


def pairwise_leaves(n):
    """Leaves of Julia's pairwise sum over n elements (pieces of <= 1024)."""
    if n <= 1024:
        return 1
    return pairwise_leaves((n + 1) // 2) + pairwise_leaves(n // 2)


def bench_kurtosis(args, cfg, eng, torch):
    """getkurtosis (src/gbtworkerfunctions.jl:197-202) over every bank of the
    config in one band launch (StatsBase recipe, Julia's pairwise Float32 mean).
    Algorithmic bytes: the window read once, plus (streamed-leaf path) the
    leaf partials written and read back by the tree merge, plus the Float64
    results."""
    win = None
    if cfg["tw"] != cfg["ntime"]:
        win = [0, cfg["nchan"], 1, 0, cfg["nif"], 1, 0, cfg["tw"], 1]
    n = cfg["nbank"] * cfg["nchan"] * cfg["nif"] * cfg["tw"]
    ncopy = cold_copies(args.cache, 4 * n)  # (cold: calls rotate over copies, >= 1 GiB)
    copies = []
    for _ in range(ncopy):
        dst = eng.band_empty(cfg["nbank"], cfg["nchan"], cfg["nif"], cfg["ntime"])
        copies.append([eng.synth(cfg["nchan"], cfg["nif"], cfg["ntime"], cfg["nfpc"],
                                 seed=10 * b + cfg["product"], kind=0, out=o)
                       for b, o in enumerate(dst)])
    banks = copies[0]
    plan = eng.kurtosis_plan(banks[0], win)
    stream = torch.cuda.current_stream()
    for w in range(max(args.warmup, ncopy)):
        eng.band_kurtosis(copies[w % ncopy], win)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(rot):
        t0 = time.perf_counter()
        e0.record(stream)
        for k in range(args.steps):
            eng.band_kurtosis(copies[k % rot], win)  # every bank in one set of launches
        e1.record(stream)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, e0.elapsed_time(e1) / args.steps

    el, ms = timed(ncopy)
    warm_ms = timed(1)[1] if ncopy > 1 else ms
    nout = cfg["nbank"] * cfg["nchan"] * cfg["nif"]
    path = plan["path"]
    reads = 2 if path == "twopass" else 1
    algo = reads * 4 * n + 8 * nout
    if path == "leaf":  # (mean, M2, M3, M4) Float64 + (sum, max, min) Float32 per leaf
        algo += 2 * 44 * nout * pairwise_leaves(cfg["tw"])
    kern = {"regs": "k_kurt_regs (one read, bit-exact recipe)",
            "mid": "k_kurt_mid (one read, register tile)",
            "leaf": "k_kurt_leaf + k_kurt_tree/k_kurt_final (one read, leaves of Julia's "
                    "pairwise sum streamed, moments merged)",
            "twopass": "k_kurt_leafsum + tree + k_kurt_pass (two reads)"}[path]
    return {"metric": "getkurtosis GB/s of filterbank input", "value": round(4 * n / ms / 1e6, 2),
            "unit": "GB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32->f64",
            "data": "synthetic (bldp_synth_f32)",
            "config": {"workload": "kurtosis over " + cfg["workload"], "name": args.config,
                       "plan": plan},
            "roofline": {"bound": "hbm", "achieved": round(algo / ms / 1e6, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo / ms / 1e6 / HBM_PEAK_GBS, 4),
                         # HBM bytes per call from the committed PMC passes (every
                         # kernel of the call; profiles/pmc_traffic.json "kurt_<cfg>")
                         "traffic": traffic_from_profile("kurt_" + args.config, cfg["nbank"]),
                         "traffic_source": traffic_from_profile("kurt_" + args.config,
                                                                cfg["nbank"], True)[1],
                         "kernel": kern, "call_ms": round(ms, 4), "bytes_per_call": algo,
                         "cache": cache_note(ncopy, 4 * n),
                         "warm": None if ncopy == 1 else {
                             "call_ms": round(warm_ms, 4),
                             "frac": round(algo / warm_ms / 1e6 / HBM_PEAK_GBS, 4)}}}


CFG5_PRODUCTS = ["cfg3", "cfg4", "cfg1"]  # 0000, 0001, 0002 single-bank geometry


def bench_host(args, eng, torch, pkg, rank=0, world=1, dist=None):
    """cfg5, the multi-band session scan streamed from pinned host memory:
    rank r takes bank r of every band, 4 bands x {0000, 0001, 0002} (12
    arrays, 24.7 GB), each through bldp_reduce_host_f32 (the Julia worker
    drop-in: host array in, reduced host array out).  At N ranks the node
    streams N banks of every band (weak scaling; N = 8 is all of cfg5: 4
    bands x 8 banks x 3 products).  Bound by PCIe (H2D), reported per GPU and
    for the node, beside the reduce kernels' HBM rate on device-resident
    copies of the same arrays."""
    import numpy as np

    dev = torch.cuda.current_device()
    bank = rank
    arrays, krate = [], []
    for band in range(4):
        for name in CFG5_PRODUCTS:
            c = CONFIGS[name]
            # seed = 1000*band + 10*bank + product
            t = eng.synth(c["nchan"], c["nif"], c["ntime"], c["nfpc"],
                          seed=1000 * band + 10 * bank + c["product"], kind=0)
            win = None if c["tw"] == c["ntime"] else [0, c["nchan"], 1, 0, c["nif"], 1, 0,
                                                      c["tw"], 1]
            if band == 0:  # the kernel's HBM rate on a device-resident copy
                eng.reduce(t, c["F"], c["T"], "sum", win)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    eng.reduce(t, c["F"], c["T"], "sum", win)
                e1.record()
                e1.synchronize()
                b = 4 * c["nif"] * (c["nchan"] * c["tw"] + (c["nchan"] // c["F"]) * (c["tw"] // c["T"]))
                krate.append((b, e0.elapsed_time(e1) / 5))
            h = torch.empty((c["ntime"], c["nif"], c["nchan"]), dtype=torch.float32,
                            pin_memory=True)
            h.copy_(t.permute(2, 1, 0))
            del t
            a = h.numpy().transpose(2, 1, 0)  # Julia-order, Fortran-contiguous, pinned
            arrays.append((a, h, c, win))
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    nbytes = sum(4 * c["nchan"] * c["nif"] * c["tw"] for _, _, c, _ in arrays)
    kern_gbs = sum(b for b, _ in krate) / (sum(ms for _, ms in krate) * 1e-3) / 1e9

    def one_pass():
        for a, _, c, win in arrays:
            eng.reduce_host(a, c["F"], c["T"], "sum", win, device=dev)

    warm = max(1, args.warmup // 5)
    for _ in range(warm):
        one_pass()
    steps = max(1, args.steps // 10)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_pass()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = (time.perf_counter() - t0) / steps
    el_max = el
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64,
                          device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el_max = float(tt[0])
    per_gpu = nbytes / el / 1e9
    node = world * nbytes / el_max / 1e9
    pg = None
    if rank == 0 and world == 1:  # the same arrays in ordinary (pageable) host memory
        pageable = [(np.asfortranarray(np.array(a, copy=True)), None, c, win)
                    for a, _, c, win in arrays[:3]]
        pbytes = sum(4 * c["nchan"] * c["nif"] * c["tw"] for _, _, c, _ in pageable)
        t1 = time.perf_counter()
        for a, _, c, win in pageable:
            eng.reduce_host(a, c["F"], c["T"], "sum", win, device=dev)
        pg = round(pbytes / (time.perf_counter() - t1) / 1e9, 2)
    return {"metric": "session scan GB/s streamed from pinned host memory (node)",
            "value": round(node, 2), "unit": "GB/s", "n_gpus": world, "steps": steps,
            "warmup": warm, "ms_per_step": round(el_max * 1e3, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (bldp_synth_f32), pinned host memory (torch pin_memory)",
            "config": {"workload": f"cfg5: rank r streams bank r of 4 bands x {{0000, 0001, "
                                   f"0002}} through bldp_reduce_host_f32 ({world} bank(s) of "
                                   f"every band on the node; 8 = all 96 arrays)",
                       "bytes_per_step_per_gpu": nbytes, "per_gpu_GBps": round(per_gpu, 2),
                       "kernel_hbm_GBps": round(kern_gbs, 1),
                       "kernel_hbm_note": "reduce kernels on device-resident copies of band "
                                          "0's three arrays (HIP events)",
                       "pageable_GBps": pg,
                       "pageable_sample": "band 0 x {0000, 0001, 0002}, ordinary numpy memory"},
            "roofline": {"bound": "pcie", "achieved": round(per_gpu, 2), "peak": 63.0,
                         "unit": "GB/s", "frac": round(per_gpu / 63.0, 4), "traffic": None,
                         "kernel": "H2D copy engine (PCIe Gen5 x16 spec 63 GB/s per GPU)"}}


def bench_decode(args, eng, torch, pkg):
    """HDF5 filter 32008 (bitshuffle + LZ4) decode on the GPU: real LZ4 chunks
    from the bitshuffle library (tests/golden/bslz4_v1.npz, a 0002-shaped
    16 x 4096 chunk), replicated to ~1 GiB of output, decoded per call with
    bldp_bslz4_decode_dev (host block-table walk + one launch + sync)."""
    import ctypes

    import numpy as np

    z = np.load(os.path.join(REPO, "tests", "golden", "bslz4_v1.npz"), allow_pickle=False)
    chunk = z["chunk_gamma_chunk_b2048"].tobytes()
    nrep = 4096
    L = pkg._lib.lib()
    comp = np.frombuffer(chunk * nrep, np.uint8)
    coff = (np.arange(nrep, dtype=np.uint64) * len(chunk))
    clen = np.full(nrep, len(chunk), np.uint64)
    raw_b = z["raw_gamma_chunk_b2048"].nbytes
    ooff = np.arange(nrep, dtype=np.uint64) * raw_b
    olen = np.full(nrep, raw_b, np.uint64)
    cdev = torch.from_numpy(comp.copy()).cuda()
    out = torch.empty(nrep * raw_b // 4, dtype=torch.float32, device="cuda")
    sp = pkg._lib.stream_ptr()

    def go():
        pkg._lib.check(L.bldp_bslz4_decode_dev(nrep, comp.ctypes.data, cdev.data_ptr(),
                                               coff.ctypes.data, clen.ctypes.data, 4,
                                               out.data_ptr(), ooff.ctypes.data, olen.ctypes.data,
                                               sp))
    for _ in range(2):
        go()
    steps = max(3, args.steps // 4)
    t0 = time.perf_counter()
    for _ in range(steps):
        go()
    el = (time.perf_counter() - t0) / steps
    ok = bool(np.array_equal(out[:raw_b // 4].cpu().numpy(),
                             z["raw_gamma_chunk_b2048"].ravel()))
    del ctypes
    return {"metric": "bitshuffle+LZ4 (HDF5 filter 32008) GPU decode, GB/s of decoded output",
            "value": round(nrep * raw_b / el / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
            "steps": steps, "warmup": 2, "ms_per_step": round(el * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8->f32",
            "data": "bitshuffle-library LZ4 chunks of synthetic 0002 power (x4096)",
            "config": {"workload": f"{nrep} chunks x {raw_b} B decoded, "
                                   f"compressed {len(chunk)} B each", "check": ok},
            "roofline": {"bound": "hbm", "achieved": round(nrep * (raw_b + len(chunk)) / el / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(nrep * (raw_b + len(chunk)) / el / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": None, "kernel": "k_bslz4 (one wave per 8 KiB block)"}}


def bench_file(args, eng, torch, pkg):
    """End to end on a compressed rawspec-style FBH5 file (HDF5 filter 32008,
    chunks (16, 1, 4096) produced by the bitshuffle library, replicated to
    1 GiB of Float32): WorkerFunctions.getdata(fname, (:,:,:); fqavby=64,
    tavby=16) = chunk reads into pinned memory + one H2D of compressed bytes
    + GPU decode + window gather + reduce.  CPU path beside it: the same file
    through the host decoder + the oracle reduce (bounded window)."""
    import numpy as np

    import __graft_entry__ as entry

    z = np.load(os.path.join(REPO, "tests", "golden", "bslz4_v1.npz"), allow_pickle=False)
    chunk = z["chunk_gamma_chunk_b2048"].tobytes()
    raw = z["raw_gamma_chunk_b2048"]  # (16, 1, 4096) C order
    nrep = 4096
    jshape = (4096, 1, 16 * nrep)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "bldp_bench_bslz4.h5")
    pkg.fbh5.write_bslz4_chunks(path, dict(foff=-187.5 / 65536, nfpc=1024), jshape,
                                (16, 1, 4096), (chunk for _ in range(nrep)))
    W = pkg.WorkerFunctions
    C = pkg.COLON
    nbytes = 4 * int(np.prod(jshape))
    got = W.getdata(path, (C, C, C), fqavby=64, tavby=16)  # warm (page cache, pinned pool)
    orc = entry.load_oracle()
    want = orc.reduce(np.asfortranarray(raw.transpose(2, 1, 0)), 64, 16)  # one chunk = one t'
    ok = bool(got.shape == (64, 1, nrep) and np.allclose(got, want, rtol=1e-5))
    steps = max(3, args.steps // 5)
    t0 = time.perf_counter()
    for _ in range(steps):
        W.getdata(path, (C, C, C), fqavby=64, tavby=16)
    el = (time.perf_counter() - t0) / steps
    tm = {}
    x = pkg.fbh5._read_window_bslz4_dev(path, (C, C, C), "cuda:0", timings=tm)
    del x
    # CPU path on a bounded window: host decode (C++) + oracle reduce
    J = pkg.JRange
    nt_cpu = 16 * 256
    t0 = time.perf_counter()
    w = pkg.fbh5.read_window_bslz4(path, (C, C, J(1, nt_cpu)), device=None)
    orc.reduce(w, 64, 16)
    cpu_el = time.perf_counter() - t0
    os.remove(path)
    return {"metric": "compressed FBH5 getdata end to end, GB/s of Float32 data",
            "value": round(nbytes / el / 1e9, 2), "unit": "GB/s", "n_gpus": 1, "steps": steps,
            "warmup": 1, "ms_per_step": round(el * 1e3, 2), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "bitshuffle-library LZ4 chunks of synthetic 0002 power",
            "config": {"workload": f"FBH5 (4096 ch x 1 IF x {16 * nrep} spectra), chunks "
                                   f"(16,1,4096) bitshuffle+LZ4, getdata fqavby=64 tavby=16",
                       "check": ok, "stages_s": {k: (round(v, 4) if isinstance(v, float) else v)
                                                 for k, v in tm.items()}},
            "roofline": {"bound": "pcie",
                         "achieved": round(tm["compressed_bytes"] / el / 1e9, 2),
                         "peak": 63.0, "unit": "GB/s",
                         "frac": round(tm["compressed_bytes"] / el / 1e9 / 63.0, 4),
                         "traffic": None,
                         "kernel": "compressed bytes moved host->device per second, end to end"},
            "cpu_baseline": {"value": round(4 * 4096 * nt_cpu / cpu_el / 1e9, 3), "unit": "GB/s",
                             "cores": 1, "kind": "port",
                             "sample": f"window (:, :, 1:{nt_cpu}): host bitshuffle/LZ4 decode "
                                       "(libbldp C++) + oracle reduce, one thread"}}


def bench_rawfile(args, eng, torch, pkg):
    """End to end on an uncompressed contiguous FBH5 file of one 0000 bank's
    geometry (2^25 ch x 1 IF x 16 spectra = 2 GiB, page cache warm):
    WorkerFunctions.getdata(fname, (:,:,:); fqavby=1024, tavby=16) = parallel
    preads into pinned slots + async H2D + one GPU reduce (filestream).  Beside
    it: the libhdf5 H5Dread + bldp_reduce_host_f32 path (the reference's read,
    reduce moved to the GPU) and the CPU path (H5Dread + oracle reduce)."""
    import numpy as np

    import __graft_entry__ as entry

    nchan, nt = 1 << 25, 16
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "bldp_bench_raw.h5")
    x = eng.synth(nchan, 1, nt, 1 << 20, seed=0, kind=0)
    a = eng.fb_to_numpy(x)
    del x
    pkg.fbh5.write(path, dict(foff=-187.5 / (1 << 20), nfpc=1 << 20), a)
    nbytes = a.nbytes
    W, C = pkg.WorkerFunctions, pkg.COLON
    orc = entry.load_oracle()
    want = orc.reduce(a, 1024, 16)
    del a
    got = W.getdata(path, (C, C, C), fqavby=1024, tavby=16)  # warm: page cache, pinned ring
    ok = bool(np.allclose(got, want, rtol=1e-5))
    steps = max(3, args.steps // 4)
    t0 = time.perf_counter()
    for _ in range(steps):
        W.getdata(path, (C, C, C), fqavby=1024, tavby=16)
    el = (time.perf_counter() - t0) / steps
    tm = {}
    runs, _, _ = pkg.filestream.plan_window((nchan, 1, nt), [0, nchan, 1, 0, 1, 1, 0, nt, 1],
                                            pkg.fbh5.raw_layout(path)[0])
    buf = pkg.filestream.read_runs_to_device(path, runs, "cuda:0", timings=tm)
    del buf
    # libhdf5 read (one thread) + host-array GPU reduce
    t0 = time.perf_counter()
    h = pkg.fbh5.read_window(path, (C, C, C))
    t_h5 = time.perf_counter() - t0
    eng.reduce_host(h, 1024, 16)
    t_old = time.perf_counter() - t0
    t0 = time.perf_counter()
    orc.reduce(h, 1024, 16)
    t_cpu = t_h5 + time.perf_counter() - t0
    del h
    os.remove(path)
    return {"metric": "uncompressed FBH5 getdata end to end, GB/s of Float32 data",
            "value": round(nbytes / el / 1e9, 2), "unit": "GB/s", "n_gpus": 1, "steps": steps,
            "warmup": 1, "ms_per_step": round(el * 1e3, 2), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic 0000-geometry bank written as an uncompressed FBH5 file",
            "config": {"workload": f"FBH5 ({nchan} ch x 1 IF x {nt} spectra, contiguous), "
                                   "getdata fqavby=1024 tavby=16", "check": ok,
                       "stream": {k: (round(v, 4) if isinstance(v, float) else v)
                                  for k, v in tm.items()},
                       "h5dread_plus_gpu_reduce_GBps": round(nbytes / t_old / 1e9, 2)},
            "roofline": {"bound": "host", "achieved": round(nbytes / el / 1e9, 2),
                         "peak": 63.0, "unit": "GB/s",
                         "frac": round(nbytes / el / 1e9 / 63.0, 4), "traffic": None,
                         "kernel": "file bytes to HBM per second (PCIe Gen5 x16 spec 63 GB/s "
                                   "as the ceiling)"},
            "cpu_baseline": {"value": round(nbytes / t_cpu / 1e9, 3), "unit": "GB/s",
                             "cores": 1, "kind": "port",
                             "sample": "the same file: libhdf5 H5Dread + oracle reduce, "
                                       "one thread"}}


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int, deadline_s: float) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes of
    this same command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU
    each) and wait for them.  Runs before anything imports torch or touches
    HIP in this process, and starts children instead of re-exec'ing; rank 0
    prints the JSON line.  Returns the exit status: 0, or the first failing
    rank's.  The ranks are polled, not waited on in order: when one exits
    non-zero (e.g. before the rendezvous or the RCCL communicator, where its
    peers would block until the process-group timeout) the others are sent
    SIGTERM, then SIGKILL after a grace period, and its status is returned.
    Ranks still running ``deadline_s`` after the start (a rank hung in a
    collective, which no exit status would ever report) are stopped the same
    way and the status is 124, as timeout(1) reports."""
    import signal
    import subprocess

    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    failed = 0
    t_end = time.monotonic() + deadline_s
    try:
        while True:
            rcs = [p.poll() for p in procs]
            failed = next((rc for rc in rcs if rc), 0)
            if failed or all(rc is not None for rc in rcs):
                break
            if time.monotonic() > t_end:
                hung = [r for r, rc in enumerate(rcs) if rc is None]
                log(f"rank(s) {hung} still running after the {deadline_s:.0f} s deadline")
                failed = 124
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        failed = 128 + signal.SIGINT
    if failed:
        log(f"stopping the ranks (status {failed})")
        for p in procs:
            if p.poll() is None:
                p.terminate()
        grace = time.monotonic() + 10.0
        for p in procs:
            try:
                p.wait(timeout=max(0.1, grace - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    # a signal-killed rank reports -SIG: exit with 128 + SIG like a shell
    return failed if failed >= 0 else 128 - failed


def rendezvous_check(args, dist, rank, world):
    """--mode rendezvous: the N-rank launch and exchange path without the GPU
    (process group, barrier, max-over-ranks timing, rank 0's JSON line), so a
    CPU-only machine can check the launch forms."""
    import torch

    dist.barrier()
    t0 = time.perf_counter()
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    g = [torch.zeros(1, dtype=torch.float64) for _ in range(world)] if rank == 0 else None
    dist.gather(torch.tensor([float(rank)], dtype=torch.float64), g, dst=0)
    dist.barrier()
    el = time.perf_counter() - t0
    r = {"metric": "bench launch rendezvous check (no GPU work)", "value": float(t[0]),
         "unit": "ranks", "n_gpus": world, "steps": 0, "warmup": 0,
         "ms_per_step": round(el * 1e3, 3), "higher_is_better": True, "scaling": "weak",
         "vs_baseline": None, "dtype": None, "data": "none",
         "config": {"workload": "rendezvous", "world_size": dist.get_world_size(),
                    "gathered_ranks": [int(x) for x in torch.cat(g)] if g else None,
                    "dist_backend": dist.get_backend()}}
    if rank == 0:
        print(json.dumps(r), flush=True)
    dist.destroy_process_group()
    return r


def bench_typed(args, eng, torch, pkg):
    """fqav and getkurtosis on 8-bit SIGPROC data (the reference's UInt8
    arrays, Blio nbits 8; src/gbtworkerfunctions.jl:173-174,197-202; and
    nbits 16, UInt16, beside it) at the
    0002 geometry: one file (65536 ch x 1 IF x 279 spectra) and the 8-file
    band, fqavby=64, sum (UInt64 results), and the kurtosis of the same data.
    Each call is prepared once per buffer (bldp_reduce_prepare /
    bldp_kurtosis_prepare: one ctypes call and the launch, as a worker
    re-reducing resident buffers pays) and the calls rotate over copies of
    the input (>= 1 GiB, cold: none in cache from the call before).  Per call:
    the GPU time of K back-to-back calls (HIP events), the kernel time alone
    (events on each launch), and the unprepared Python call (engine.reduce /
    engine.kurtosis) for comparison."""
    import numpy as np

    rng = np.random.default_rng(0)
    out = {}
    HipEvent = pkg._lib.HipEvent
    sp = int(torch.cuda.current_stream().cuda_stream)
    for label, nb, dt in (("0002 file", 1, np.uint8), ("0002 band", 8, np.uint8),
                          ("0002 file u16", 1, np.uint16), ("0002 band u16", 8, np.uint16)):
        # C order [t][i][c]; UInt16: SIGPROC nbits 16
        a = rng.integers(0, np.iinfo(dt).max, (279, 1, 65536 * nb), dtype=dt, endpoint=True)
        ncopy = cold_copies(args.cache, a.nbytes)  # cold: calls rotate over >= 1 GiB of copies
        xs = [torch.from_numpy(a).cuda().permute(2, 1, 0)  # Julia-order (65536*nb, 1, 279)
              for _ in range(ncopy)]
        preps = {"reduce": [eng.PreparedReduce(x, 64, 1, "sum") for x in xs],
                 "kurtosis": [eng.PreparedKurtosis(x) for x in xs]}
        calls = {"reduce": lambda x: eng.reduce(x, 64, 1, "sum"),
                 "kurtosis": lambda x: eng.kurtosis(x)}
        rec = out[label] = {"input_bytes": int(a.nbytes), "cache": cache_note(ncopy, a.nbytes)}
        for what, pl in preps.items():
            for w in range(max(args.warmup, ncopy)):
                pl[w % ncopy].launch(sp)
            torch.cuda.synchronize()
            e0, e1 = HipEvent(timing=True, fence=False), HipEvent(timing=True, fence=False)
            evs = [(HipEvent(timing=True, fence=False), HipEvent(timing=True, fence=False))
                   for _ in range(args.steps)]

            def timed(rot, fn):
                e0.record(sp)
                t0 = time.perf_counter()
                for k in range(args.steps):
                    fn(k % rot)
                host = (time.perf_counter() - t0) / args.steps
                e1.record(sp)
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / args.steps, host * 1e3

            ms, host_ms = timed(ncopy, lambda c: pl[c].launch(sp))
            warm_ms = timed(1, lambda c: pl[0].launch(sp))[0] if ncopy > 1 else ms
            for k in range(args.steps):  # the kernel alone: events on each launch
                pl[k % ncopy].launch_timed(sp, *evs[k])
            torch.cuda.synchronize()
            kern = sorted(x.elapsed_time(y) for x, y in evs)[args.steps // 2]
            py_ms = timed(ncopy, lambda c: calls[what](xs[c]))[0]  # the unprepared Python call
            nbytes = a.nbytes + (8 * (65536 * nb // 64) * 279 if what == "reduce"
                                 else 8 * 65536 * nb)
            rec[what] = {"ms_per_call": round(ms, 4), "kernel_ms": round(kern, 4),
                         "host_enqueue_ms_per_call": round(host_ms, 4),
                         "GBps_in_plus_out": round(nbytes / ms / 1e6, 1),
                         "GBps_of_input": round(a.nbytes / ms / 1e6, 1),
                         "frac": round(nbytes / ms / 1e6 / HBM_PEAK_GBS, 4),
                         "warm_ms_per_call": round(warm_ms, 4),
                         "unprepared_python_ms_per_call": round(py_ms, 4)}
            for p_ in pl:
                p_.close()
    f = out["0002 band"]["reduce"]
    return {"metric": "fqav GB/s on UInt8 SIGPROC data (0002 band geometry, fqavby=64, sum)",
            "value": f["GBps_in_plus_out"], "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": f["ms_per_call"], "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u8->u64",
            "data": "synthetic uniform 0..255", "config": {"workload": "typed reduce", **out},
            "roofline": {"bound": "hbm", "achieved": f["GBps_in_plus_out"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": f["frac"],
                         "traffic": traffic_from_profile("typed_band", 1),
                         "traffic_source": traffic_from_profile("typed_band", 1, True)[1],
                         "kernel": "k_reduce_typed_vec16 (8-file band, one call per step)",
                         "cache": out["0002 band"]["cache"],
                         "warm": {"ms_per_call": f["warm_ms_per_call"],
                                  "frac": round(f["GBps_in_plus_out"] * f["ms_per_call"]
                                                / f["warm_ms_per_call"] / HBM_PEAK_GBS, 4)}}}


def verify_band(cfg, eng, torch, dist, banks, mine, nb, run_step, rank, world, use_pg):
    """The timed path checked on its own result, after the timed region: this
    rank's banks are regenerated in place as integer data (bldp_synth_f32
    kind 1, values 0..255, so every Float32 sum of F*T <= 65536 of them is
    exact in any order), ``run_step()`` runs one step exactly as timed
    (prepared reduce into the rank's slice; N > 1: the exchange to the root and
    its stitch) and returns the root's stitched band.  Every rank computes, from
    its own inputs, each bank's window total and a few spot groups (Float64,
    exact); the root gathers them and compares every bank's vcat slot of the
    product bit for bit (src/gbt.jl:75-78,103: reduce(vcat, fetch.(futures))).
    Returns (ok, detail) on the root, (None, None) elsewhere."""
    F, T = cfg["F"], cfg["T"]
    nco, ni, nto = cfg["nchan"] // F, cfg["nif"], cfg["tw"] // T
    for b, v in zip(mine, banks):
        eng.synth(cfg["nchan"], cfg["nif"], cfg["ntime"], cfg["nfpc"],
                  seed=7919 + 10 * b + cfg["product"], kind=1, out=v)
    spots = [(0, 0, 0), (nco // 2, ni - 1, nto // 2), (nco - 1, ni - 1, nto - 1)]
    expect = []
    for b, v in zip(mine, banks):
        row = [v[:, :, :nto * T].sum(dtype=torch.float64)]
        for k, i, t in spots:
            row.append(v[k * F:(k + 1) * F, i, t * T:(t + 1) * T].sum(dtype=torch.float64))
        expect.append(torch.stack(row))
    expect = torch.stack(expect)  # (banks of this rank, 1 + spots)
    torch.cuda.synchronize()
    product = run_step()
    torch.cuda.synchronize()
    if world > 1:
        nccl = dist.get_backend() == "nccl"
        mine_t = expect if nccl else expect.cpu()
        allx = [torch.empty_like(mine_t) for _ in range(world)] if rank == 0 else None
        dist.gather(mine_t, allx, dst=0)
        if rank != 0:
            return None, None
        expect = torch.cat([x.to(product.device) for x in allx])
    if tuple(product.shape) != (nb * nco, ni, nto):
        return False, f"product shape {tuple(product.shape)} != {(nb * nco, ni, nto)}"
    bad = []
    for b in range(nb):
        slot = product[b * nco:(b + 1) * nco]
        got = [slot.sum(dtype=torch.float64)] + [slot[k, i, t].double() for k, i, t in spots]
        got = torch.stack(got).cpu()
        want = expect[b].cpu()
        if not torch.equal(got, want):
            bad.append({"bank": b, "got": got.tolist(), "want": want.tolist()})
    detail = (f"integer data (bldp_synth_f32 kind 1), one step of the timed path; {nb} banks' "
              f"vcat slots: window total + {len(spots)} spot groups each, bit-exact")
    return not bad, (detail if not bad else {"mismatch": bad[:4], "check": detail})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-read-probe", action="store_true",
                    help="skip the box pure-read reference (roofline.box_read_probe)")
    ap.add_argument("--mode", default="reduce",
                    choices=["reduce", "kurtosis", "host", "decode", "file", "rawfile",
                             "rendezvous", "typed"])
    ap.add_argument("--local-banks", type=int, default=None,
                    help="N=1 only: reduce just this many banks per launch, i.e. one rank's "
                         "share of an N-GPU run (for per-launch PMC profiles)")
    ap.add_argument("--band-alloc", default="slab", choices=["per-bank", "slab"],
                    help="banks as separate allocations or as views of one slab")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo only to rehearse the N-rank path on one GPU")
    ap.add_argument("--exchange", default="native", choices=["native", "torch"],
                    help="nccl backend: the per-step gather through libbldp_hip's "
                         "bldp_band_gather_f32 on a stream of its own (native) or "
                         "torch.distributed.gather (torch)")
    ap.add_argument("--pipeline", action="store_true",
                    help="N=1: run the N>1 exchange anyway (a one-rank process group, "
                         "RCCL gather + stitch of every step) to exercise it on one GPU")
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="untimed launches for this long before the warmup steps (GPU clocks)")
    ap.add_argument("--cache", default="auto", choices=["auto", "cold", "warm"],
                    help="cold: rotate launches over copies of the input totalling >= 1 GiB "
                         "(auto: when a launch reads < 1 GiB); warm figures are reported "
                         "beside the cold ones")
    ap.add_argument("--plan-option", action="append", default=[], metavar="NAME=VALUE",
                    help="override a planner choice (bldp_plan_option; A/B runs only)")
    ap.add_argument("--rank-deadline", type=float, default=900.0,
                    help="N>1 without a launcher: seconds after which ranks still running "
                         "(e.g. hung in a collective) are stopped and bench.py exits 124")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the integer-data check of one step after the timed region")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: this process only starts the N ranks (no torch, no HIP here)
        sys.exit(spawn_ranks(args.gpus, args.rank_deadline))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.mode == "rendezvous":
        # BENCH_RENDEZVOUS_FAIL_RANK=r: rank r exits with status 3 before the
        # rendezvous, as a rank that dies before init_process_group does (the
        # fail-fast test of spawn_ranks; rendezvous mode only)
        if os.environ.get("BENCH_RENDEZVOUS_FAIL_RANK") == str(rank):
            log(f"rank {rank}: injected failure before the rendezvous")
            sys.exit(3)
        # BENCH_RENDEZVOUS_HANG_RANK=r: rank r never reaches the rendezvous (a
        # rank hung in a collective; the deadline test of spawn_ranks)
        if os.environ.get("BENCH_RENDEZVOUS_HANG_RANK") == str(rank):
            log(f"rank {rank}: injected hang before the rendezvous")
            while True:
                time.sleep(60)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("gloo")
        return rendezvous_check(args, dist, rank, world)

    import __graft_entry__ as entry

    pkg = entry.load_package()
    eng = pkg.engine
    for o in args.plan_option:
        name, _, val = o.partition("=")
        pkg._lib.check(pkg._lib.lib().bldp_plan_option(name.encode(), int(val), None),
                       "bldp_plan_option")
    local = local % max(1, torch.cuda.device_count())  # gloo rehearsal: ranks share GPUs
    torch.cuda.set_device(local)
    use_pg = world > 1 or args.pipeline
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    cfg = CONFIGS[args.config]
    run_info = {"dist_backend": args.dist_backend if use_pg else None,
                "exchange": (args.exchange if args.dist_backend == "nccl" else "torch")
                if use_pg else None,
                "world_size": dist.get_world_size() if use_pg else 1,
                "device_count": torch.cuda.device_count()}
    if args.mode == "host":
        r = bench_host(args, eng, torch, pkg, rank, world, dist if use_pg else None)
        r["config"].update(run_info)
        if rank == 0:
            print(json.dumps(r), flush=True)
        if use_pg:
            dist.barrier()
            dist.destroy_process_group()
        return r
    if args.mode != "reduce":
        if world != 1:
            raise SystemExit("--mode kurtosis/typed/decode/file/rawfile are single-GPU measurements")
        r = (bench_kurtosis(args, cfg, eng, torch) if args.mode == "kurtosis"
             else bench_typed(args, eng, torch, pkg) if args.mode == "typed"
             else bench_decode(args, eng, torch, pkg) if args.mode == "decode"
             else bench_file(args, eng, torch, pkg) if args.mode == "file"
             else bench_rawfile(args, eng, torch, pkg))
        r["config"].update(run_info)
        print(json.dumps(r), flush=True)
        return r
    nb = cfg["nbank"]
    if nb % world:
        raise SystemExit(f"{nb} banks do not shard over {world} GPUs")
    mine = list(pkg.band.banks_for_rank(nb, rank, world)) if nb >= world else [0]
    if args.local_banks:
        if world != 1 or nb % args.local_banks:
            raise SystemExit("--local-banks: N=1 only, and it must divide the bank count")
        mine = mine[:args.local_banks]
        nb = len(mine)  # the job is this share of the band
    win = None
    if cfg["tw"] != cfg["ntime"]:
        win = [0, cfg["nchan"], 1, 0, cfg["nif"], 1, 0, cfg["tw"], 1]  # idxs=(:, :, 1:tw)

    nco, ni, nto = cfg["nchan"] // cfg["F"], cfg["nif"], cfg["tw"] // cfg["T"]
    read_b = 4 * cfg["nchan"] * cfg["nif"] * cfg["tw"]
    write_b = 4 * nco * ni * nto
    bytes_step = nb * (read_b + write_b)          # whole band (all ranks)
    bytes_launch = len(mine) * (read_b + write_b)  # this rank's single reduce launch
    # --cache cold (auto: launches below 1 GiB): the steps rotate over `ncopy`
    # distinct copies of the rank's banks, >= 1 GiB in all, so no launch finds
    # its input in the 256 MB Infinity Cache the previous launches filled (a
    # 71 MB cfg1 window re-read launch after launch mostly would: its pure
    # read passes 8 TB/s); warm figures beside them
    ncopy = cold_copies(args.cache, bytes_launch)

    log(f"rank {rank}/{world}: generating banks {mine} of {args.config} on device"
        + (f" ({ncopy} copies, cold cache)" if ncopy > 1 else ""))
    # the rank's banks: views of one HBM slab (engine.band_empty), or separate
    # allocations (--band-alloc per-bank, 2.4% slower on MI355X)
    copies = []
    for _ in range(ncopy):
        dst = eng.band_empty(len(mine), cfg["nchan"], cfg["nif"], cfg["ntime"]) \
            if args.band_alloc == "slab" else [None] * len(mine)
        copies.append([eng.synth(cfg["nchan"], cfg["nif"], cfg["ntime"], cfg["nfpc"],
                                 seed=10 * b + cfg["product"], kind=0, out=o)
                       for b, o in zip(mine, dst)])
        del dst  # the banks keep the slab alive (freed before the CPU baseline)
    banks = copies[0]
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    # this rank's slice of the band; N > 1: two slots, the RCCL gather of step
    # k (to rank 0, over xGMI) overlaps the reduce of step k+1
    native_x = use_pg and args.dist_backend == "nccl" and args.exchange == "native"
    if not use_pg:
        pipe = None
    elif native_x:
        pipe = pkg.band.NativeBandPipeline(len(mine) * nco, ni, nto, device=f"cuda:{local}")
    else:
        pipe = pkg.band.BandPipeline(len(mine) * nco, ni, nto, device=f"cuda:{local}",
                                     gather_single=args.pipeline)
    out = eng.fb_empty(len(mine) * nco, ni, nto) if pipe is None else None

    # the reduce prepared once per output slot (bldp_band_reduce_prepare_f32):
    # a step costs the host one ctypes call + the kernel launch
    sp = int(stream.cuda_stream)
    preps = {}

    def step(ev0=None, ev1=None, copy=0):
        slot = pipe.begin() if pipe else 0
        prep = preps.get((copy, slot))
        if prep is None:
            dst = pipe.local(slot) if pipe else out
            prep = preps[copy, slot] = eng.PreparedBandReduce(copies[copy], cfg["F"], cfg["T"],
                                                              "sum", win, out=dst)
        if ev0 is not None:  # the events ride on the kernel dispatch itself
            prep.launch_timed(sp, ev0, ev1)
        else:
            prep.launch(sp)
        return pipe.exchange(slot) if pipe else prep.out  # root: the stitched band

    # clock settle: the GPU's clocks ramp under sustained load, so the W
    # warmup steps are preceded by untimed launches until --settle-ms of GPU
    # time has passed (the 0002 band's 86 us kernel: 85.8 us after 5 warmup
    # launches, 83.9 us after 300, profiles/r04/bench_cfg2_warmup_r04e.json)
    # (the reduce alone, into an output of its own: ranks may settle for
    # different counts without unbalancing the exchange's collectives)
    settle = 0
    if args.settle_ms > 0:
        sprep = eng.PreparedBandReduce(banks, cfg["F"], cfg["T"], "sum", win)
        t_settle = time.perf_counter()
        while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
            for _ in range(8):
                sprep.launch(sp)
            settle += 8
            torch.cuda.synchronize()
        sprep.close()
        del sprep
    for w in range(max(args.warmup, ncopy)):
        step(copy=w % ncopy)
    if pipe:
        pipe.drain()
    torch.cuda.synchronize()
    # timing-only events without the system-scope fence, carried by the
    # reduce's own dispatches (bldp_reduce_launch_timed).  Even so, an event
    # pair costs a launch ~4 us of command-processor time (tools/gap_probe.py:
    # cfg1 11.4 us a step bare, 15.0 with events on every launch), so the
    # timed steps carry only the two that span them: the first launch's start
    # and the last one's end.  The per-launch kernel time comes from K more
    # launches right after, each carrying its own pair (what rocprofv3's
    # kernel trace reports).
    HipEvent = pkg._lib.HipEvent
    evs = [(HipEvent(timing=True, fence=False), HipEvent(timing=True, fence=False))
           for _ in range(args.steps)]
    sp0, sp1, sx0, sx1 = (HipEvent(timing=True, fence=False) for _ in range(4))
    K = args.steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        c = k % ncopy
        if K == 1:
            step(sp0, sp1, copy=c)
        elif k == 0:
            step(sp0, sx1, copy=c)
        elif k == K - 1:
            step(sx0, sp1, copy=c)
        else:
            step(copy=c)
    host_ms = (time.perf_counter() - t0) * 1e3 / K  # enqueue cost per step
    if pipe:
        pipe.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    span_ms = sp0.elapsed_time(sp1) / K  # first kernel's start to last one's end, per launch
    for k in range(K):  # the kernel pass
        step(*evs[k], copy=(K + k) % ncopy)
    if pipe:
        pipe.drain()
    torch.cuda.synchronize()
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / K
    warm_ms = kern_ms
    if ncopy > 1:  # the same K launches on one copy: the warm (cache-resident) figure
        for k in range(K):
            step(*evs[k], copy=0)
        if pipe:
            pipe.drain()
        torch.cuda.synchronize()
        warm_ms = sum(a.elapsed_time(b) for a, b in evs) / K
    if world > 1:
        t = torch.tensor([el, kern_ms, span_ms, warm_ms], dtype=torch.float64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern_ms, span_ms, warm_ms = float(t[0]), float(t[1]), float(t[2]), float(t[3])
    verified, verify_detail = None, None
    if not args.no_verify:
        def one_step():
            res = step(copy=0)
            if pipe:
                pipe.drain()
            return res
        verified, verify_detail = verify_band(cfg, eng, torch, dist, banks, mine, nb, one_step,
                                              rank, world, use_pg)
    ms_step = el * 1e3 / args.steps
    path = eng.plan(banks[0], cfg["F"], cfg["T"], "sum", win)["path"] if banks else None
    kernel_name = {"interleaved": "k_reduce_il", "vector": "k_reduce_vec",
                   "narrow": "k_reduce_narrow", "tile": "k_reduce_tile",
                   "scalar": "k_reduce_scalar"}.get(path, path) + \
        f" ({len(mine)}-bank launch)"
    value = bytes_step / (ms_step * 1e-3) / 1e9
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = traffic_from_profile(args.config, len(mine), with_source=True)

    ndev = torch.cuda.device_count()
    if not pipe:
        parallelism = f"{len(mine)} bank(s) x 1 GPU, single-launch band reduce + stitch"
    elif args.dist_backend == "nccl":
        via = ("ncclGather through libbldp_hip (bldp_band_gather_f32) on its own stream"
               if native_x else "torch.distributed.gather")
        parallelism = (f"{len(mine)} bank(s)/GPU x {world} GPU(s), RCCL (nccl backend) gather "
                       f"over xGMI + stitch ({via}); the gather of step k overlaps the reduce "
                       "of step k+1")
    else:
        parallelism = (f"REHEARSAL, not a scaling number: {world} ranks on {ndev} GPU(s), gloo "
                       f"backend (CPU transport) gather + stitch, {len(mine)} bank(s)/rank")
    result = None
    if rank == 0:
        # this box's pure-read rate for a buffer of the launch's bytes
        # (tools/hbm_probe.hip, the pure read of tools/mix_ceiling.hip): HBM rates
        # differ box to box by several percent, so the reduce is also set
        # beside what a kernel that only reads reaches on the same GPU
        probe = None
        if not args.no_read_probe:
            preps.clear()
            torch.cuda.empty_cache()
            sys.path.insert(0, os.path.join(REPO, "tools"))
            import hbm_probe

            probe = hbm_probe.read_probe(bytes_launch, stream=stream, pkg=pkg, copies=ncopy)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            preps.clear()  # (they hold the banks)
            del banks, copies
            torch.cuda.empty_cache()
            log("cpu baseline (oracle port) ...")
            cpu = cpu_baseline(cfg, args.cpu_seconds, eng, torch)
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: gamma(2, 5e8) x per-coarse-channel bandpass x DC spike, "
                    "generated on device (bldp_synth_f32); no published reference number",
            "config": {"workload": cfg["workload"], "name": args.config, "nbank": nb,
                       "nchan": cfg["nchan"], "nif": cfg["nif"], "ntime": cfg["tw"],
                       "fqavby": cfg["F"], "tavby": cfg["T"],
                       "band_alloc": args.band_alloc,
                       "parallelism": parallelism,
                       "bytes_per_step": bytes_step, **run_info},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kernel_name,
                         "kernel_ms": round(kern_ms, 4),
                         "kernel_ms_source": "per-launch dispatch events over K launches after "
                                             "the timed region",
                         "span_ms_per_launch": round(span_ms, 4),
                         "bytes_per_launch": bytes_launch,
                         "box_read_probe": probe,
                         "frac_of_box_read": probe and round(achieved / probe["GBps"], 4),
                         "cache": cache_note(ncopy, bytes_launch),
                         "warm": None if ncopy == 1 else {
                             "kernel_ms": round(warm_ms, 4),
                             "achieved": round(bytes_launch / (warm_ms * 1e-3) / 1e9, 1),
                             "frac": round(bytes_launch / (warm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                           4),
                             "note": "the same launches on one copy, its input left in the "
                                     "Infinity Cache by the launch before"}},
            "host_enqueue_ms_per_step": round(host_ms, 4),
            "settle_launches": settle,
            "verified": verified,
            "verify": verify_detail,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if use_pg:
        dist.barrier()
        if native_x:
            pipe.close()
        dist.destroy_process_group()
    if verified is False:
        log(f"VERIFY FAILED: {verify_detail}")
        sys.exit(5)
    return result


if __name__ == "__main__":
    main()
