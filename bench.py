#!/usr/bin/env python3
"""Benchmark: batched 1D c2c FFT N=2^20 (BASELINE.json configs[1]) on MI355X.

A "step" is one hsfft_exec_batched over the per-GPU batch (4096 x 2^20 complex f64, inputs
already resident in HBM).  Multi-GPU: one process per GPU; each rank transforms its own 4096
rows (weak scaling, no data-path collective -- the path shards by batch index); rank 0 prints
one JSON line with the max-over-ranks time.  `bench.py --gpus N` started without a launcher
starts the N rank processes itself (torch.distributed.run as a child process, before anything
touches the GPU) and exits with their status; under a launcher (torch.distributed.run sets
WORLD_SIZE) WORLD_SIZE must equal N.

Other configs: --config c1 (one N=1024 fft_exec on HOST buffers: latency, next to the
reference timed in the same run), c3 (12600 x 65536), c4 (Bluestein 99991 x 8192), c5 (r2c
2^22 x 32768 over the job, chunked per GPU).

roofline: achieved = algorithmic bytes of the whole step (32 B per complex
sample for c2c) / the event-timed step time, i.e. the transform as a whole, every launch of
the step included; `pass_frac` lists the same figure per launch of a multi-launch step.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "mixed-radix-fast-fourier-transform_amd")
sys.path.insert(0, PKG)

import hsfft  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)

CONFIGS = {
    # name: (kind, N, per-GPU batch, seed, description)
    "c1": ("latency", 1024, 1, 0x5EED0001, "one N=1024 c2c forward fft_exec on host buffers (drop-in API)"),
    "c2": ("c2c", 1 << 20, 4096, 0x5EED0002, "batched c2c N=2^20, batch=4096 per GPU, fp64"),
    "c3": ("c2c", 12600, 65536, 0x5EED0003, "mixed-radix c2c N=12600, batch=65536 per GPU, fp64"),
    "c4": ("c2c", 99991, 8192, 0x5EED0004, "Bluestein c2c N=99991, batch=8192 per GPU, fp64"),
    "c5": ("r2c", 1 << 22, 4096, 0x5EED0005, "r2c N=2^22, 4096 rows per GPU (32768 over 8 GPUs), fp64"),
}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


class Comm:
    """Barrier + max-reduce across ranks.  The FFT path has no exchange step, so the only
    communication is control: gloo over TCP (no GPU buffers are involved)."""

    def __init__(self, ws):
        self.ws = ws
        self.dist = None
        if ws > 1:
            import torch
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist, self.torch = dist, torch

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, v):
        if not self.dist:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, v):
        """all ranks' values of a float, in rank order"""
        if not self.dist:
            return [v]
        t = self.torch.tensor([float(v)], dtype=self.torch.float64)
        out = [self.torch.zeros_like(t) for _ in range(self.ws)]
        self.dist.all_gather(out, t)
        return [float(x.item()) for x in out]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: N rank processes (one per GPU) under
    torch.distributed.run, started as CHILD processes of this one -- which has not touched the
    GPU and never replaces itself -- on 127.0.0.1; returns their exit status."""
    import subprocess
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *argv]
    return subprocess.call(cmd, env=env)


def row_range(rank, per_rank_batch):
    """Weak-scaling shard: rank r transforms global rows [r*B, (r+1)*B) -- the batch index is
    the only thing split across GPUs (no data-path collective)."""
    return rank * per_rank_batch, (rank + 1) * per_rank_batch


def rank_fields(comm, ws, wall_s, steps, ev_ms_per_step, bytes_per_step):
    """Per-rank breakdown of the timed region: every rank's
    own wall ms per step (between the same barriers), its event-timed ms per step and the
    algorithmic bytes it moved / its event time against ONE GPU's peak, plus the aggregate --
    the bytes of all ranks / the max-over-ranks wall time -- against ws x the peak.  Collective
    calls: every rank must call this."""
    walls = comm.gather(wall_s / steps * 1e3)
    evs = comm.gather(ev_ms_per_step)
    per = []
    for r in range(ws):
        ach = bytes_per_step / (evs[r] / 1e3) / 1e9 if evs[r] > 0 else 0.0
        per.append({"rank": r, "ms_per_step": round(walls[r], 4), "event_ms_per_step": round(evs[r], 4),
                    "achieved": round(ach, 3), "frac": round(ach / HBM_PEAK_GBS, 6)})
    agg = bytes_per_step * ws / (max(walls) / 1e3) / 1e9 if max(walls) > 0 else 0.0
    return per, {"achieved": round(agg, 3), "peak": HBM_PEAK_GBS * ws, "unit": "GB/s",
                 "frac": round(agg / (HBM_PEAK_GBS * ws), 6),
                 "basis": f"algorithmic bytes of all {ws} ranks / the max-over-ranks wall ms per step"}


def dry_run(args, comm, ws, rank):
    """The multi-rank control path without a GPU (CPU tests under gloo): every rank transforms
    its own rows of a small c2c batch with the CPU oracle, timed with the same barrier /
    max-over-ranks protocol; rank 0 prints the JSON line plus every rank's row range."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import numpy as np

    import hsfft_testlib as T
    n, batch = args.dry_n, args.batch or 4
    r0, r1 = row_range(rank, batch)
    x = T.complex_input(n, 0x5EED0002, batch=batch, row0=r0).reshape(batch, n)
    lib = T.oracle()
    p = lib.orc_plan_create(n, 1, 0)
    y = np.zeros_like(x)
    run = lambda: lib.orc_exec_batch(p, T.ptr(x), T.ptr(y), batch, 1)  # noqa: E731
    for _ in range(args.warmup):
        run()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    comm.barrier()
    local = time.perf_counter() - t0
    wall = comm.max(local)
    rows = comm.gather(r0)
    checks = comm.gather(float(np.abs(y).sum()))
    lib.orc_plan_destroy(p)
    ms = wall / args.steps * 1e3
    # the same per-rank / aggregate fields as a GPU line (the CPU "event" time is the wall time)
    per, agg = rank_fields(comm, ws, local, args.steps, local / args.steps * 1e3, n * batch * 32)
    if rank == 0:
        out = {"metric": f"dry run: c2c N={n} on the CPU oracle (no GPU)", "value": round(
            n * batch * ws / (ms / 1e3) / 1e9, 6), "unit": "GSamples/s", "n_gpus": ws, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "dry_run": True, "per_rank_batch": batch, "row_starts": [int(r) for r in rows],
            "rank_checksums": checks, "per_rank": per,
            "roofline": {"bound": "hbm", "unit": "GB/s", "aggregate": agg}}
        if not args.no_cpu_baseline:  # rank 0, after the timed region, as on the GPU line
            out["cpu_baseline"] = cpu_baseline(("c2c", n, batch, 0x5EED0002, ""), seconds_target=0.5)
        print(json.dumps(out), flush=True)


def host_cores():
    """CPU cores this process may use: the affinity mask, capped by a cgroup CPU quota
    (a GPU box shows the whole machine in os.cpu_count() but grants a share of it)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    use = min(aff, quota) if quota else aff
    return max(1, use), {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": quota, "cpu_model": model}


def cpu_baseline(cfg, seconds_target=15.0):
    """The reference (oracle/_ref, compiled from the unmodified sources) timed on ALL host
    cores available to this process (one plan per thread) over a bounded sample: `sample`
    distinct transforms, swept `reps` times so that the timed region is ~seconds_target of
    wall time.  Falls back to the oracle restatement ('port') when the reference build is
    absent."""
    kind, n, _, seed, _ = cfg
    threads, hostinfo = host_cores()
    ref_so = os.path.join(REPO, "oracle", "_ref", "libhsref.so")
    sample = {("c2c", 1 << 20): 128, ("c2c", 12600): 8192, ("c2c", 99991): 64, ("r2c", 1 << 22): 32}.get((kind, n), 64)
    sample = max(sample, threads)  # at least one transform per thread
    if os.path.exists(ref_so):
        L = ctypes.CDLL(ref_so)
        L.hsref_time_batch_reps.restype = ctypes.c_double
        L.hsref_time_batch_reps.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint64, ctypes.c_int]
        real = 1 if kind == "r2c" else 0
        t1 = L.hsref_time_batch_reps(n, 1, real, sample, threads, seed, 1)  # calibration sweep
        reps = max(1, min(1000, int(seconds_target / max(t1, 1e-6))))
        secs = L.hsref_time_batch_reps(n, 1, real, sample, threads, seed, reps)
        src = "reference"
    else:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import numpy as np

        import hsfft_testlib as T
        lib = T.oracle()
        if kind == "r2c":
            x = T.real_input(n, seed, batch=sample).reshape(sample, n)
            h = lib.orc_real_create(n, 1, 0)
            y = np.zeros((sample, n), dtype=np.complex128)
            go = lambda: lib.orc_r2c_batch(h, T.ptr(x), T.ptr(y), sample, threads)  # noqa: E731
        else:
            x = T.complex_input(n, seed, batch=sample).reshape(sample, n)
            h = lib.orc_plan_create(n, 1, 0)
            y = np.zeros_like(x)
            go = lambda: lib.orc_exec_batch(h, T.ptr(x), T.ptr(y), sample, threads)  # noqa: E731
        t0 = time.perf_counter()
        go()
        t1 = time.perf_counter() - t0
        reps = max(1, min(1000, int(seconds_target / max(t1, 1e-6))))
        t0 = time.perf_counter()
        for _ in range(reps):
            go()
        secs = time.perf_counter() - t0
        (lib.orc_real_destroy if kind == "r2c" else lib.orc_plan_destroy)(h)
        src = "port"
    return {"value": round(n * sample * reps / secs / 1e9, 6), "unit": "GSamples/s", "cores": threads, "kind": src,
            "sample": f"{sample} distinct transforms of N={n} ({kind}) x {reps} sweeps, {threads} threads, "
                      f"one plan per thread, {secs:.2f} s wall", **hostinfo}


def traffic_entry(cfg_name):
    try:
        with open(os.path.join(REPO, "profiles", "pmc_traffic.json")) as f:
            return json.load(f).get(cfg_name) or {}
    except (OSError, ValueError):
        return {}


def read_traffic(cfg_name, batch):
    """HBM bytes of one whole step (every kernel of the step, per launch count) from the
    committed PMC summary (rocprofv3 FETCH_SIZE x2 [gfx950 calibration] + WRITE_SIZE, per
    MI355X_MICROARCH.md §HBM), valid only for the batch and schedule it was measured at."""
    ent = traffic_entry(cfg_name)
    if not ent or ent.get("batch", CONFIGS[cfg_name][2]) != batch:
        return None
    return ent.get("hbm_bytes_per_step")


def bench_c1(args, comm, ws, rank):
    """BASELINE config 1: ONE N=1024 forward c2c through the drop-in fft_exec on host buffers
    (ref highSpeedFFT.c:1920; the reference takes ~9 us on one core).  Per-call latency is
    timed call by call (ctypes overhead ~1 us included) and reported as the median; the
    reference (oracle/_ref) is timed on one host core in the same run."""
    import numpy as np
    kind, n, _, seed, desc = CONFIGS["c1"]
    plan = hsfft.Plan(n, 1)
    dx = hsfft.DeviceBuffer(n * 16)
    hsfft.fill_complex(dx, n, seed, 0)
    x = dx.to_array(np.complex128, n)
    y = np.zeros_like(x)
    L = hsfft.lib()
    px, py = x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p)
    for _ in range(max(args.warmup, 20)):
        L.fft_exec(plan.ptr, px, py)
    iters = max(args.steps, 200)
    lat = []
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):  # through the Python binding: reported beside, not the value
        t = time.perf_counter()
        L.fft_exec(plan.ptr, px, py)
        lat.append(time.perf_counter() - t)
    wall = comm.max(time.perf_counter() - t0)
    lat.sort()
    # the value: a C loop of fft_exec calls, as the reference's own number is taken
    us = (ctypes.c_double * 4)()
    hsfft.check(L.hsfft_time_exec_host(plan.ptr, px, py, 1, max(iters, 2000), max(args.warmup, 50), us),
                "time_exec_host")
    med_us = us[0]
    out = {"metric": "latency of one N=1024 c2c fft_exec on host buffers (BASELINE config 1)",
           "value": round(med_us, 2), "unit": "us", "n_gpus": ws, "steps": iters, "warmup": max(args.warmup, 20),
           "ms_per_step": round(wall / iters * 1e3, 5), "higher_is_better": False, "scaling": "replicas only",
           "vs_baseline": None, "dtype": "f64 (complex128)", "data": "synthetic (splitmix64 uniform [-1,1))",
           "config": {"workload": desc, "N": n, "per_gpu_batch": 1, "global_batch": ws,
                      "parallelism": "replicas only"},
           "value_basis": "median of per-call latencies in a C loop (hsfft_time_exec_host), as the reference is timed",
           "latency_us": {"p10": round(us[1], 2), "median": round(us[0], 2), "p90": round(us[2], 2),
                          "mean": round(us[3], 2)},
           "latency_us_ctypes": {"p10": round(lat[len(lat) // 10] * 1e6, 2), "median": round(lat[len(lat) // 2] * 1e6, 2),
                                 "p90": round(lat[len(lat) * 9 // 10] * 1e6, 2)}}
    if rank == 0 and not args.no_cpu_baseline:
        cb = c1_cpu_baseline(seed)
        if cb:
            out["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(out), flush=True)
    dx.free()


def c1_c_loop(nthreads=1, iters=2000, warmup=50):
    """BASELINE config 1 timed as the reference is: fft_exec of N=1024 on host buffers in a C loop
    (hsfft_time_exec_host: no binding overhead between calls; `nthreads` fresh threads after
    warm-up threads that exited).  Returns (median, p10, p90, aggregate us per transform)."""
    import numpy as np
    L = hsfft.lib()
    p1 = hsfft.Plan(1024, 1)
    x = np.ascontiguousarray(np.exp(1j * np.arange(1024.0)))
    y = np.zeros_like(x)
    us = (ctypes.c_double * 4)()
    hsfft.check(L.hsfft_time_exec_host(p1.ptr, x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p),
                                       nthreads, iters, warmup, us), "time_exec_host")
    p1.close()
    return [float(v) for v in us]


def c1_latency(iters=300, warmup=20):
    """median latency of one N=1024 forward c2c fft_exec on host buffers (drop-in API)"""
    import numpy as np
    L = hsfft.lib()
    p1 = hsfft.Plan(1024, 1)
    x = np.ascontiguousarray(np.exp(1j * np.arange(1024.0)))
    y = np.zeros_like(x)
    px, py = x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p)
    for _ in range(warmup):
        L.fft_exec(p1.ptr, px, py)
    lat = []
    for _ in range(iters):
        t = time.perf_counter()
        L.fft_exec(p1.ptr, px, py)
        lat.append(time.perf_counter() - t)
    lat.sort()
    p1.close()
    return lat


def c1_threads(nthreads=8, iters=200):
    """N=1024 fft_exec on host buffers from `nthreads` host threads at once, one plan shared
    (the reference's fft_exec is reentrant): mean wall time per transform over all threads"""
    import threading
    import numpy as np
    L = hsfft.lib()
    p1 = hsfft.Plan(1024, 1)
    xs = [np.ascontiguousarray(np.exp(1j * (np.arange(1024.0) + t))) for t in range(nthreads)]
    ys = [np.zeros_like(x) for x in xs]

    def work(t, k):
        px, py = xs[t].ctypes.data_as(ctypes.c_void_p), ys[t].ctypes.data_as(ctypes.c_void_p)
        for _ in range(k):
            L.fft_exec(p1.ptr, px, py)
    ths = [threading.Thread(target=work, args=(t, 20)) for t in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    ths = [threading.Thread(target=work, args=(t, iters)) for t in range(nthreads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    wall = time.perf_counter() - t0
    p1.close()
    return wall / (nthreads * iters) * 1e6


def c1_cpu_baseline(seed=0x5EED0001, reps=200000):
    """the reference's fft_exec for N=1024 on ONE host core (its own single-thread design)"""
    ref_so = os.path.join(REPO, "oracle", "_ref", "libhsref.so")
    if not os.path.exists(ref_so):
        return None
    R = ctypes.CDLL(ref_so)
    R.hsref_time_batch_reps.restype = ctypes.c_double
    R.hsref_time_batch_reps.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint64, ctypes.c_int]
    secs = R.hsref_time_batch_reps(1024, 1, 0, 1, 1, seed, reps)
    return {"value": round(secs / reps * 1e6, 3), "unit": "us", "cores": 1, "kind": "reference",
            "sample": f"{reps} back-to-back fft_exec calls of N=1024 on one core, {secs:.2f} s"}


PLACE_MIN_GBS = 5900.0  # copy rate below which an output buffer counts as a slow placement


def place_output(din, dout, tries=3):
    """Physical-placement check of the output buffer, BEFORE the input is generated.

    On this pool a fresh 64 GiB hipMalloc lands in one of two kinds of physical memory: writes
    into it run at ~7.0 TB/s or ~5.75 TB/s (reads ~6.3 either way; the stream copy 6.0 vs 5.3
    TB/s), and which one a buffer gets is a lottery of the allocation, not of the kernels
    (tools/experiments/alloc_rate.hip).  Every FFT pass writes its
    output buffer, so a slow placement costs ~10 % of c2 (81 vs 90 GSamples/s, same box).
    The probe is a 16-B stream copy din -> dout (what a write-bound pass sees); if dout is
    slow (below 5.9 TB/s: fast placements copy at 5.95-6.15, slow ones at 5.3-5.8), dout -> din is
    tried (roles swapped: din is only read), then up to `tries` fresh
    output buffers.  The kept buffers and every probe rate are reported in the JSON line.
    Returns (din, dout, record)."""
    def rate(src, dst):
        """the slowest 4-GiB slice of dst: placement is decided per physical chunk, not per
        buffer -- a 64 GiB output whose whole-buffer copy rate passed once held a slow half
        that made every second c5 split launch 34 % slower (profiles/r04b_c5_walk_halves.txt)"""
        sl = 4 << 30
        n = min(src.nbytes, sl) // 16 * 16
        worst = None
        for off in range(0, dst.nbytes - 15, sl):
            m = min(n, (dst.nbytes - off) // 16 * 16)
            ms = hsfft.bench_copy(src, hsfft.DeviceView(dst, off), m, 2)
            r = 2 * m * 2 / (ms / 1e3) / 1e9
            worst = r if worst is None or r < worst else worst
        return round(worst, 1)

    rec = {"probe": "16-B stream copy into every 4-GiB slice of the output buffer, slowest slice, GB/s", "min_gbs": PLACE_MIN_GBS, "copy_gbs": []}
    r = rate(din, dout)
    rec["copy_gbs"].append(r)
    if r >= PLACE_MIN_GBS:
        return din, dout, rec
    if din.nbytes == dout.nbytes:
        r2 = rate(dout, din)
        rec["copy_gbs"].append(r2)
        if r2 >= PLACE_MIN_GBS:
            rec["swapped"] = True
            return dout, din, rec
    best, best_r, extra = dout, r, []
    for _ in range(tries):
        try:
            cand = hsfft.DeviceBuffer(dout.nbytes)
        except hsfft.HsfftError:
            break
        rc = rate(din, cand)
        rec["copy_gbs"].append(rc)
        extra.append(cand)
        if rc > best_r:
            best, best_r = cand, rc
        if rc >= PLACE_MIN_GBS:
            break
    for b in [dout] + extra:
        if b is not best:
            b.free()
    rec["reallocations"] = len(extra)
    return din, best, rec


def probe_placement(din, dout):
    """Diagnostic only (the buffers are not changed): the copy rate into every 4-GiB slice of the
    output buffer.  Round 3 selected buffers by this kind of probe; round 4 found it does not
    predict the r2c split's time (a first allocation whose slices all copied at 5.46-5.74 TB/s ran
    c5 at 105.8 GSamples/s, the re-allocated 'best' one at 87.6: profiles/r04c_*), so the bench
    line now times the buffers as first allocated and only reports the probe."""
    sl = 4 << 30
    n = min(din.nbytes, sl) // 16 * 16
    rates = []
    for off in range(0, dout.nbytes - 15, sl):
        m = min(n, (dout.nbytes - off) // 16 * 16)
        ms = hsfft.bench_copy(din, hsfft.DeviceView(dout, off), m, 2)
        rates.append(round(2 * m * 2 / (ms / 1e3) / 1e9, 1))
    return {"probe": "16-B stream copy into each 4-GiB slice of the output buffer, GB/s (diagnostic; buffers "
                     "kept as first allocated)", "slice_copy_gbs": rates}


def other_configs(steps=10, warmup=2, cpu=True, cpu_seconds=8.0):
    """The other BASELINE configs, each at its full per-GPU workload, timed in the same run as
    the headline (one rank): `steps` steps between HIP events on the library stream after
    `warmup` untimed ones (the wall clock of the same steps is reported beside), inputs
    generated in HBM; each with its roofline fraction, its PMC traffic (profiles/
    pmc_traffic.json, when measured at this batch) and the reference timed on the host cores
    over a bounded sample (`cpu_seconds` per config).  c1 is the median latency of single
    host-buffer fft_exec calls beside the reference on one core."""
    out = {}
    lat = c1_latency()
    one, eight = c1_c_loop(1, 2000, 50), c1_c_loop(8, 500, 20)
    out["c1"] = {"value": round(one[0], 2), "unit": "us", "workload": CONFIGS["c1"][4],
                 "value_basis": "median of per-call latencies in a C loop (hsfft_time_exec_host), as the reference "
                                "is timed", "higher_is_better": False, "steps": 2000,
                 "latency_us": {"p10": round(one[1], 2), "p90": round(one[2], 2), "mean": round(one[3], 2)},
                 "threads8_us_per_transform": round(eight[3], 2),
                 "threads8_basis": "8 fresh C threads after 8 warm-up threads exited, 500 calls each, one shared plan: "
                                   "wall time / 4000 transforms",
                 "latency_us_ctypes": {"median": round(lat[len(lat) // 2] * 1e6, 2),
                                       "p10": round(lat[len(lat) // 10] * 1e6, 2),
                                       "p90": round(lat[len(lat) * 9 // 10] * 1e6, 2)},
                 "threads8_us_per_transform_python": round(c1_threads(), 2)}
    if cpu:
        out["c1"]["cpu_baseline"] = c1_cpu_baseline()
    L = hsfft.lib()
    for name in ("c3", "c4", "c5"):
        kind, n, batch, seed, desc = CONFIGS[name]
        bufs = {}
        if kind == "c2c":
            plan = hsfft.Plan(n, 1)
            bufs["in"], bufs["out"] = hsfft.DeviceBuffer(n * batch * 16), hsfft.DeviceBuffer(n * batch * 16)
            fill = lambda: hsfft.fill_complex(bufs["in"], n * batch, seed, 0)  # noqa: E731
            run = lambda: hsfft.exec_batched(plan, bufs["in"], bufs["out"], batch)  # noqa: E731
            timed = lambda k: hsfft.time_batched(plan, bufs["in"], bufs["out"], batch, k)[0]  # noqa: E731
        else:
            plan = hsfft.RealPlan(n, 1)
            chunk = min(batch, max(1, (32 << 30) // (n * 16)))  # 512-row output chunks (32 GiB), as the headline
            bufs["in"], bufs["out"] = hsfft.DeviceBuffer(n * batch * 8), hsfft.DeviceBuffer(chunk * n * 16)
            fill = lambda: hsfft.fill_real(bufs["in"], n * batch, seed, 0)  # noqa: E731

            def run():
                for c0 in range(0, batch, chunk):
                    hsfft.check(L.hsfft_r2c_batched(plan.ptr, ctypes.c_void_p(bufs["in"].ptr + c0 * n * 8),
                                                    ctypes.c_void_p(bufs["out"].ptr), min(chunk, batch - c0)), "r2c")

            def timed(k):  # every chunk of the step, `k` steps, event-timed per chunk call
                tot = 0.0
                for c0 in range(0, batch, chunk):
                    sub = hsfft.DeviceView(bufs["in"], c0 * n * 8)
                    tot += hsfft.time_r2c_batched(plan, sub, bufs["out"], min(chunk, batch - c0), k)
                return tot

        def measure():
            for _ in range(warmup):
                run()
            hsfft.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                run()
            hsfft.synchronize()
            return (time.perf_counter() - t0) / steps * 1e3, timed(steps) / steps

        # the buffers as first allocated (what a caller's plain hipMalloc gets): no selection
        place = probe_placement(bufs["in"], bufs["out"])
        fill()
        wall_ms, ev_ms = measure()
        din, dout = bufs["in"], bufs["out"]
        bps = 32 if kind == "c2c" else 24
        alg = n * batch * bps
        ach = alg / (ev_ms / 1e3) / 1e9
        ent = traffic_entry(name)
        out[name] = {"value": round(n * batch / (ev_ms / 1e3) / 1e9, 3), "unit": "GSamples/s",
                     "value_basis": "buffers as first allocated (plain hipMalloc, no placement selection)",
                     "ms_per_step": round(ev_ms, 3), "wall_ms_per_step": round(wall_ms, 3), "steps": steps,
                     "warmup": warmup, "frac": round(ach / HBM_PEAK_GBS, 4),
                     "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": read_traffic(name, batch),
                                  "algorithmic_bytes": alg,
                                  "kernel": (ent.get("kernel", "") or "").replace("void ", "") or None},
                     "placement": place,
                     "workload": desc}
        din.free()
        dout.free()
        plan.close()
        if cpu:
            out[name]["cpu_baseline"] = cpu_baseline(CONFIGS[name], seconds_target=cpu_seconds)
    return out


def bench_convolve(args, comm, ws, rank):
    """batched linear convolution: r2c (compact, split fused) x2, spectral product on bins
    0..P/2, c2r, scale, 'full' window copy -- the GPU form of convolve.c:74-214"""
    L = hsfft.lib()
    n = m = 1 << 20
    rows = args.convolve
    da = hsfft.DeviceBuffer(rows * n * 8)
    db = hsfft.DeviceBuffer(rows * m * 8)
    hsfft.fill_real(da, rows * n, 0x5EED0006, row_range(rank, rows)[0] * n)
    hsfft.fill_real(db, rows * m, 0x5EED0007, row_range(rank, rows)[0] * m)
    clen = n + m - 1
    P = 1 << (clen - 1).bit_length()
    dout = hsfft.DeviceBuffer(rows * clen * 8)

    def run():
        ln = L.hsfft_convolve_batched(b"full", b"linear", ctypes.c_void_p(da.ptr), n, ctypes.c_void_p(db.ptr), m,
                                      ctypes.c_void_p(dout.ptr), rows)
        if ln != clen:
            raise SystemExit(f"convolve_batched returned {ln}: {L.hsfft_last_error()}")
    for _ in range(args.warmup):
        run()
    hsfft.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    hsfft.synchronize()
    comm.barrier()
    wall = comm.max(time.perf_counter() - t0)
    ms = wall / args.steps * 1e3
    if rank == 0:
        print(json.dumps({"metric": "GSamples/s (batched linear convolution, padded length P x rows per second)",
                          "value": round(rows * P * ws / (ms / 1e3) / 1e9, 3), "unit": "GSamples/s", "n_gpus": ws,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                          "data": "synthetic (splitmix64 uniform [-1,1), generated in HBM)",
                          "config": {"workload": f"convolve full/linear, {n} x {m} -> {clen} (P = {P}), {rows} rows",
                                     "per_gpu_batch": rows, "global_batch": rows * ws,
                                     "parallelism": f"batch-sharded x{ws} (no collective)"}}), flush=True)
    for d in (da, db, dout):
        d.free()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="override per-GPU batch (development only)")
    ap.add_argument("--n", type=int, default=0, help="override the transform length (development only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="wall-time target of the cpu_baseline leg's timed sweeps (tests shorten it)")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="c2, one rank: skip timing BASELINE configs c1, c3, c4, c5 after the headline")
    ap.add_argument("--r2c-compact", action="store_true",
                    help="c5 only: hsfft_r2c_batched_compact (N/2+1 bins per row) instead of the reference layout")
    ap.add_argument("--c2r", action="store_true",
                    help="c5 only: time hsfft_c2r_batched (the inverse real path, SURVEY.md §8f item 2) instead of r2c")
    ap.add_argument("--convolve", type=int, default=0, metavar="ROWS",
                    help="time hsfft_convolve_batched (SURVEY.md §8f item 1): ROWS linear 'full' convolutions "
                         "of 2^20-sample pairs (P = 2^21); value = padded samples P x ROWS per second")
    ap.add_argument("--dry-run", action="store_true", help="multi-rank control path on the CPU oracle (tests)")
    ap.add_argument("--dump-rows", default="",
                    help="c2c / r2c: after the timed steps, save the first and last output row of this rank's "
                         "shard (r2c: of the step's last output chunk) with their global row indices to "
                         "DIR/rank<r>.npz (multi-rank parity test)")
    ap.add_argument("--dry-n", type=int, default=1024)
    ap.add_argument("--no-finalize", action="store_true",
                    help="skip hsfft_finalize() before exit (diagnostics: the library's teardown is on by default)")
    ap.add_argument("--host-rows", type=int, default=0,
                    help="also time hsfft_exec_batched_host on this many HOST-resident rows (PCIe-inclusive "
                         "rate, reported as host_pipeline; never the headline value)")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))  # before any GPU call in this process
    ws, rank, local = dist_env()
    if ws != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}: launch one rank per GPU "
                         f"(--nproc-per-node must equal --gpus)")
    comm = Comm(ws)
    try:
        bench_main(args, comm, ws, rank, local)
    finally:
        if not args.dry_run and not args.no_finalize and hsfft._lib is not None:
            # release every device object before the process exits (a pending launch error of
            # this thread would be reported here; say so, without masking an earlier exception)
            if hsfft.lib().hsfft_finalize() != 0:
                print(f"bench.py: hsfft_finalize: {hsfft.lib().hsfft_last_error().decode()}", file=sys.stderr)
        comm.close()


def bench_main(args, comm, ws, rank, local):
    if args.dry_run:
        dry_run(args, comm, ws, rank)
        return
    L = hsfft.lib()
    ndev = hsfft.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible")
    hsfft.check(L.hsfft_set_device(local % ndev), "set_device")
    if args.convolve:
        bench_convolve(args, comm, ws, rank)
        return
    if args.config == "c1":
        bench_c1(args, comm, ws, rank)
        return

    cfg = CONFIGS[args.config]
    kind, n, batch, seed, desc = cfg
    if args.r2c_compact and kind == "r2c":
        desc += " [compact N/2+1 output, hsfft_r2c_batched_compact]"
    if args.c2r and kind == "r2c":
        desc = desc.replace("r2c", "c2r", 1) + " [hsfft_c2r_batched, N/2+1 bins read per row]"
    if args.n:
        desc += f" [N overridden to {args.n}: not the BASELINE workload]"
        n = args.n
    if args.batch:
        desc += f" [per-GPU batch overridden to {args.batch}: not the BASELINE workload]"
        batch = args.batch
    samples = n * batch
    chunk = batch
    place = None
    if kind == "c2c":
        plan = hsfft.Plan(n, 1)
        din = hsfft.DeviceBuffer(samples * 16)
        dout = hsfft.DeviceBuffer(samples * 16)
        fill = lambda: hsfft.fill_complex(din, samples, seed, row_range(rank, batch)[0] * n)  # noqa: E731
        run = lambda: hsfft.exec_batched(plan, din, dout, batch)  # noqa: E731
        bytes_per_sample = 32  # read 16 B + write 16 B
        dtype = "f64 (complex128)"
    elif args.c2r:
        plan = hsfft.RealPlan(n, -1)
        # spectra in (N complex per row, bins 0..N/2 read), N reals out: the real output of all
        # rows stays resident, the spectra are one chunk re-read per chunk of rows
        chunk = min(batch, max(1, (64 << 30) // (n * 16)))
        dout = hsfft.DeviceBuffer(samples * 8)
        din = hsfft.DeviceBuffer(chunk * n * 16)
        hsfft.fill_complex(din, chunk * n, seed, 0)
        fill = None

        def run():
            for c0 in range(0, batch, chunk):
                cb = min(chunk, batch - c0)
                hsfft.check(L.hsfft_c2r_batched(plan.ptr, ctypes.c_void_p(din.ptr),
                                                ctypes.c_void_p(dout.ptr + c0 * n * 8), cb), "c2r_batched")
        bytes_per_sample = 16  # read 8 B (N/2+1 bins) + write 8 B
        dtype = "f64"
    else:
        plan = hsfft.RealPlan(n, 1)
        # the whole per-GPU input stays resident (4096 x 2^22 x 8 B = 128 GiB); the mirrored
        # N-bin output (16 B per real sample) of all rows would not fit next to it in 288 GB,
        # so the step writes it chunk by chunk into one output buffer a consumer would drain:
        # 512 rows (32 GiB) per call, the library's own chunk of the inner intermediate, so the
        # placement check can afford up to three fresh output buffers next to the input
        chunk = min(batch, max(1, (32 << 30) // (n * 16)))
        din = hsfft.DeviceBuffer(samples * 8)
        orow = (n // 2 + 1) if args.r2c_compact else n
        dout = hsfft.DeviceBuffer(chunk * orow * 16)
        fill = lambda: hsfft.fill_real(din, samples, seed, row_range(rank, batch)[0] * n)  # noqa: E731
        fn = hsfft.lib().hsfft_r2c_batched_compact if args.r2c_compact else hsfft.lib().hsfft_r2c_batched

        def run():
            for c0 in range(0, batch, chunk):
                cb = min(chunk, batch - c0)
                hsfft.check(fn(plan.ptr, ctypes.c_void_p(din.ptr + c0 * n * 8), ctypes.c_void_p(dout.ptr), cb),
                            "r2c_batched")
        # read 8 B + write 16 B of the mirrored output (compact: 8 B of the N/2+1 bins)
        bytes_per_sample = 16 if args.r2c_compact else 24
        dtype = "f64"
    hsfft.synchronize()

    def timed_steps():
        """W untimed warmup steps, then exactly K steps between barrier + synchronize on both
        sides; the max over ranks of the wall time"""
        for _ in range(args.warmup):
            run()
        hsfft.synchronize()
        comm.barrier()
        hsfft.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        hsfft.synchronize()
        comm.barrier()
        local = time.perf_counter() - t0
        return comm.max(local), local

    # the buffers as first allocated -- what a caller's plain hipMalloc gets; no placement
    # selection (probe_placement only reports the output buffer's slice copy rates)
    if fill is not None:
        place = probe_placement(din, dout)
        fill()
        hsfft.synchronize()
    wall, wall_local = timed_steps()

    # HIP-event timing on the library stream (what the kernels take) + per-pass breakdown
    npass = 0
    pass_ms = []
    if kind == "c2c":
        ev_ms, pms = hsfft.time_batched(plan, din, dout, batch, max(1, args.steps))
        npass = plan.num_passes()
        pass_ms = [p for p in pms[:npass] if p > 0]
    elif args.r2c_compact or args.c2r:
        ev_ms = wall * 1e3
    else:
        ev_ms = hsfft.time_r2c_batched(plan, din, dout, chunk, max(1, args.steps)) * (batch / chunk)
    ev_local_ms = ev_ms / max(1, args.steps)
    ev_step_ms = comm.max(ev_local_ms)

    ms_per_step = wall / args.steps * 1e3
    value = samples * ws / (ms_per_step / 1e3) / 1e9
    out = {
        "metric": "GSamples/s + achieved HBM GB/s, batched 1D c2c FFT N=2^20 at 1/2/4/8 MI355X"
        if args.config == "c2" else f"GSamples/s ({desc})",
        "value": round(value, 3),
        "unit": "GSamples/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (splitmix64 uniform [-1,1), generated in HBM)",
        "config": {"workload": desc, "N": n, "per_gpu_batch": batch, "global_batch": batch * ws,
                   "parallelism": f"batch-sharded x{ws} (no collective)", "passes": npass,
                   **({"output_chunk_rows": chunk} if chunk != batch else {})},
        "achieved_hbm_gbs": round(samples * bytes_per_sample * ws / (ms_per_step / 1e3) / 1e9, 1),
        "event_ms_per_step": round(ev_step_ms, 4),
    }
    if place:
        out["placement"] = place
    out["value_basis"] = "buffers as first allocated (plain hipMalloc, no placement selection)"
    # the transform as a whole: algorithmic bytes of the step / event-timed step time
    ach = samples * bytes_per_sample / (ev_step_ms / 1e3) / 1e9
    ent = traffic_entry(args.config)
    kern = ent.get("kernel", "").replace("void ", "") if ent.get("batch") == batch else ""
    launches = f"{max(npass, 1)} launch(es)"
    if kind == "c2c" and plan.header()["lt"] != 0 or args.config == "c4":  # Bluestein
        launches = ("one persistent launch (bxc::k_bxcd) per 65536 rows"
                    if os.environ.get("HSFFT_BLUE_XCD", "8") != "0" else "3 launches per 1024-row chunk")
    out["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": read_traffic(args.config, batch),
                       "algorithmic_bytes": samples * bytes_per_sample,
                       "basis": f"whole step: {bytes_per_sample} B x N x batch / event-timed step time, "
                                f"{launches} of the step",
                       "kernel": kern or f"{launches} per step"}
    if ws > 1:  # every rank's own numbers, and the whole job's bytes against ws x the peak
        out["per_rank"], out["roofline"]["aggregate"] = rank_fields(comm, ws, wall_local, args.steps, ev_local_ms,
                                                                    samples * bytes_per_sample)
    if pass_ms:
        out["roofline"]["pass_ms"] = [round(p, 4) for p in pass_ms]
        out["roofline"]["pass_frac"] = [round(samples * bytes_per_sample / (p / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                                        for p in pass_ms]
    # (before the copy benchmark below overwrites dout)
    if args.dump_rows and not args.c2r:
        import numpy as np
        g0 = row_range(rank, batch)[0]
        if kind == "c2c":
            picks = sorted({0, batch - 1})
            rows = np.stack([dout.to_array(np.complex128, n, r * n * 16) for r in picks])
        else:  # r2c: the output buffer holds the step's last chunk of rows
            c0 = (batch - 1) // chunk * chunk
            orow = (n // 2 + 1) if args.r2c_compact else n
            picks = sorted({c0, batch - 1})
            rows = np.stack([dout.to_array(np.complex128, orow, (r - c0) * orow * 16) for r in picks])
        os.makedirs(args.dump_rows, exist_ok=True)
        np.savez(os.path.join(args.dump_rows, f"rank{rank}.npz"), rows=rows,
                 global_rows=np.array([g0 + r for r in picks]), n=n, seed=seed, world=ws, kind=kind)
    # practical HBM ceiling on this device: a 16-B-per-lane stream copy of the same buffers
    nbytes = min(din.nbytes, dout.nbytes) // 16 * 16
    cms = hsfft.bench_copy(din, dout, nbytes, 5)
    out["stream_copy_gbs"] = round(2 * nbytes * 5 / (cms / 1e3) / 1e9, 1)
    if args.host_rows and kind == "c2c":
        import numpy as np
        hb = min(args.host_rows, batch)
        hx = din.to_array(np.complex128, hb * n).reshape(hb, n)
        hy = np.empty_like(hx)
        hsfft.exec_batched_host(plan, hx, hy)  # warm-up (plan state, staging slots)
        t0 = time.perf_counter()
        hsfft.exec_batched_host(plan, hx, hy)
        hs = time.perf_counter() - t0
        out["host_pipeline"] = {"rows": hb, "gsamples_s": round(hb * n / hs / 1e9, 3),
                                "pcie_gbs": round(2 * hx.nbytes / hs / 1e9, 1),
                                "note": "host (pageable numpy) rows in and out, upload/transform/download overlapped; "
                                        "PCIe-inclusive, not the headline value"}
    if rank == 0 and not args.no_cpu_baseline and not args.c2r:
        # rank 0, after every rank's timed region (at N > 1 too: north_star wants the reference
        # timed on the host cores in the same run next to the 1/2/4/8-GPU numbers)
        out["cpu_baseline"] = cpu_baseline(cfg, seconds_target=args.cpu_seconds)
    if ws == 1 and args.config == "c2" and not args.batch and not args.n and not args.no_other_configs:
        din.free()
        dout.free()
        out["other_configs"] = other_configs(cpu=not args.no_cpu_baseline)
    if rank == 0:
        print(json.dumps(out), flush=True)
    din.free()
    dout.free()


if __name__ == "__main__":
    main()
