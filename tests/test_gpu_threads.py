"""Reentrancy of the drop-in API on the MI355X: several host threads call the reference's
entry points at once (the reference's mixed-radix fft_exec is const on its plan and uses no
globals, highSpeedFFT.c:1920-1942 / 318-1629; r2c/c2r/convolve malloc per call, real.c:87-88,
convolve.c:104-154).  ctypes releases the GIL around every foreign call, so the threads below
really are inside libhsfft together.

Every output is compared BIT-EXACT with the oracle (CPU restatement pinned to the reference).
"""
import threading

import numpy as np
import pytest

import hsfft_testlib as T

import hsfft

pytestmark = pytest.mark.gpu

NTHREADS = 8
ITERS = 6
# ten distinct padded lengths P (2^7 .. 2^16): more than the 8 cached plan pairs, so cache
# entries are evicted and rebuilt while other threads are still using theirs
CONV = [(40 + 7 * k, (1 << (k + 6)) - 40 - 7 * k + 1) for k in range(10)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if hsfft.device_count() < 1:
        pytest.skip("no GPU")
    hsfft.lib().hsfft_set_device(0)
    yield
    hsfft.synchronize()


def _conv_ref(a, b, typ=b"full"):
    o = np.zeros(2 * (a.size + b.size) + 8)
    ln = T.oracle().orc_convolve(typ, b"linear", T.ptr(a), a.size, T.ptr(b), b.size, T.ptr(o), 0)
    return o[:ln].copy()


def test_eight_threads_shared_plan_r2c_and_convolve():
    L = hsfft.lib()
    n_c = 12600                     # mixed radix 3/5/7/8 (config 3's length), ONE shared plan
    shared = hsfft.Plan(n_c, 1)
    n_r = 1 << 14                   # real path: one shared real plan
    rplan = hsfft.RealPlan(n_r, 1)
    n_b = 97                        # Bluestein: one plan per thread (the reference's rule)

    xs = [T.complex_input(n_c, 0x7000 + t) for t in range(NTHREADS)]
    ref_c = [T.oracle_c2c(x, 1) for x in xs]
    rs = [T.real_input(n_r, 0x7100 + t) for t in range(NTHREADS)]
    ref_r = [T.oracle_r2c(r, 1) for r in rs]
    bs = [T.complex_input(n_b, 0x7200 + t) for t in range(NTHREADS)]
    ref_b = [T.oracle_c2c(b, -1) for b in bs]
    conv_in = []
    for k, (n, m) in enumerate(CONV):
        a, b = T.real_input(n, 0x7300 + k), T.real_input(m, 0x7400 + k)
        conv_in.append((a, b, _conv_ref(a, b)))
    assert len({1 << (n + m - 2).bit_length() for n, m in CONV}) >= 9

    errors = []
    start = threading.Barrier(NTHREADS)

    def worker(t):
        try:
            L.hsfft_set_device(0)
            bplan = hsfft.Plan(n_b, -1)
            start.wait()
            for it in range(ITERS):
                y = np.zeros(n_c, dtype=np.complex128)
                L.fft_exec(shared.ptr, T.ptr(xs[t]), T.ptr(y))
                if not T.bits_equal(y, ref_c[t]):
                    errors.append(("c2c", t, it, T.mismatches(y, ref_c[t])))
                Y = np.zeros(n_r, dtype=np.complex128)
                L.fft_r2c_exec(rplan.ptr, T.ptr(rs[t]), T.ptr(Y))
                if not T.bits_equal(Y, ref_r[t]):
                    errors.append(("r2c", t, it, T.mismatches(Y, ref_r[t])))
                z = bplan.exec(bs[t])
                if not T.bits_equal(z, ref_b[t]):
                    errors.append(("bluestein", t, it))
                k = (t * 3 + it) % len(CONV)
                a, b, ref = conv_in[k]
                o = np.zeros(ref.size + 8)
                ln = L.fft_convolve(b"full", b"linear", T.ptr(a), a.size, T.ptr(b), b.size, T.ptr(o))
                if ln != ref.size or not T.bits_equal(o[:ln], ref):
                    errors.append(("convolve", t, it, k, ln))
            bplan.close()
        except Exception as e:  # pragma: no cover - reported below
            errors.append(("exception", t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(NTHREADS)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not any(x.is_alive() for x in th), "a worker thread did not finish"
    assert not errors, errors[:10]


def test_threads_batched_device_api_distinct_plans():
    """the extension API from several threads: each thread its own device buffers, the
    plans shared (2^20 two-pass, 4096, 12600 whole-row kernel), results bit-exact"""
    sizes = [1 << 20, 4096, 12600, 1 << 16]
    plans = {n: hsfft.Plan(n, 1) for n in sizes}
    errors = []

    def worker(t):
        try:
            hsfft.lib().hsfft_set_device(0)
            n = sizes[t % len(sizes)]
            rows = 2 if n == 1 << 20 else 5
            x = T.complex_input(n, 0x7500 + t, batch=rows).reshape(rows, n)
            din = hsfft.DeviceBuffer.from_array(x)
            dout = hsfft.DeviceBuffer(x.nbytes)
            for _ in range(3):
                hsfft.exec_batched(plans[n], din, dout, rows)
                hsfft.synchronize()
                y = dout.to_array(np.complex128).reshape(rows, n)
                if not T.bits_equal(y, T.oracle_c2c(x, 1)):
                    errors.append((t, n))
            din.free()
            dout.free()
        except Exception as e:  # pragma: no cover
            errors.append(("exception", t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(NTHREADS)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not any(x.is_alive() for x in th)
    assert not errors, errors


def test_exec_multi_threads_single_device():
    """hsfft_exec_multi runs one host thread per device (here ndev = 1: the shard thread
    path and its error propagation)"""
    import ctypes
    n, rows = 4096, 6
    x = T.complex_input(n, 0x7600, batch=rows).reshape(rows, n)
    p = hsfft.Plan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(x.nbytes)
    ins = (ctypes.c_void_p * 1)(din.ptr)
    outs = (ctypes.c_void_p * 1)(dout.ptr)
    assert hsfft.lib().hsfft_exec_multi(p.ptr, ins, outs, rows, 1) == 0
    y = dout.to_array(np.complex128).reshape(rows, n)
    assert T.bits_equal(y, T.oracle_c2c(x, 1))
    assert hsfft.lib().hsfft_exec_multi(p.ptr, ins, outs, rows, 99) < 0   # more devices than exist


def test_thread_generations_recycle_resources():
    """threads that come and go recycle the per-thread resources of the
    lock-free small path (stream, page-locked slots, completion word) -- parked at exit, adopted
    by the next thread, never created or destroyed on a live caller's path (round 5 reaped dead
    threads' objects on a new thread's first call: +52 % per threaded call).  Three generations
    of 8 threads call the drop-in fft_exec on one shared 1024-point plan (BASELINE config 1):
    every output bit-exact vs the oracle, and the three generations create at most 8 streams.
    Then generations whose threads make exactly ONE call, then two: a recycled completion word
    must continue its previous owner's sequence (round 6: a new owner restarting at 1 found 1
    already in the word and copied its output before its kernel had run)."""
    L = hsfft.lib()
    n = 1024
    plan = hsfft.Plan(n, 1)
    xs = [T.complex_input(n, 0x7700 + t) for t in range(NTHREADS)]
    refs = [T.oracle_c2c(x, 1) for x in xs]
    errors = []
    s0 = L.hsfft_thread_streams_created()

    def worker(t, gen, calls):
        try:
            L.hsfft_set_device(0)
            for it in range(calls):
                y = np.zeros(n, dtype=np.complex128)
                L.fft_exec(plan.ptr, T.ptr(xs[t]), T.ptr(y))
                if not T.bits_equal(y, refs[t]):
                    errors.append((gen, t, it, T.mismatches(y, refs[t])))
        except Exception as e:  # pragma: no cover
            errors.append(("exception", gen, t, repr(e)))

    for gen, calls in enumerate([40, 40, 40, 1, 2, 1, 3]):
        start = threading.Barrier(NTHREADS)

        def run(t, gen=gen, start=start, calls=calls):
            start.wait()
            worker(t, gen, calls)

        th = [threading.Thread(target=run, args=(t,)) for t in range(NTHREADS)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=120)
        assert not any(x.is_alive() for x in th)
    made = L.hsfft_thread_streams_created() - s0
    assert not errors, errors[:10]
    assert made <= NTHREADS, f"seven generations of {NTHREADS} threads created {made} streams"
    plan.close()


@pytest.mark.parametrize("nthreads", [1, 8])
def test_time_exec_host_c_loop(nthreads):
    """hsfft_time_exec_host (bench.py's c1 value since round 6: fft_exec in a C loop, as the
    reference is timed): warm-up threads then fresh timed threads; the output is bit-exact and
    the statistics are ordered"""
    import ctypes
    L = hsfft.lib()
    n = 1024
    p = hsfft.Plan(n, 1)
    x = T.complex_input(n, 0x7800)
    y = np.zeros(n, dtype=np.complex128)
    us = (ctypes.c_double * 4)()
    assert L.hsfft_time_exec_host(p.ptr, T.ptr(x), T.ptr(y), nthreads, 100, 5, us) == 0
    assert T.bits_equal(y, T.oracle_c2c(x, 1))
    assert 0 < us[1] <= us[0] <= us[2] and us[3] > 0
    p.close()
