"""GPU parity of the hot-path kernel families against the oracle:

* pf::k_firstq / pf::k_b512 (csrc/hsfft_pass_pf.h): the two passes of 2^20 (BASELINE config
  2) and the [8,8,8,8] first pass of 2^21 (config 5's inner c2c);
* bxc::k_bxcd (csrc/hsfft_blue_xcd.h): Bluestein M = 2^18 (config 4) as one persistent launch
  with in-launch hand-offs, checked on small odd batches, under uneven load (per-phase
  random delays) and at the FULL config-4 size on every output word;
* bpf::k_bfirst / k_bmid / k_blast (csrc/hsfft_blue_pf.h): the three-launch Bluestein path
  (the persistent launch's fallback).

Tolerance: bit-exact (0 ulp) against the oracle (the CPU restatement pinned to the reference)
and against the other schedules of the same transform.
"""
import numpy as np
import pytest

import hsfft_testlib as T

import hsfft

pytestmark = pytest.mark.gpu

N = 1 << 20


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if hsfft.device_count() < 1:
        pytest.skip("no GPU")
    hsfft.lib().hsfft_set_device(0)
    yield
    hsfft.synchronize()


def _run(x, sgn):
    batch = x.shape[0]
    p = hsfft.Plan(N, sgn)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(x.nbytes)
    hsfft.exec_batched(p, din, dout, batch)
    hsfft.synchronize()
    y = dout.to_array(np.complex128).reshape(x.shape)
    din.free()
    dout.free()
    p.close()
    return y


_cache = {}


def _oracle(x, sgn, key):
    k = (key, sgn)
    if k not in _cache:
        _cache[k] = T.oracle_c2c(x, sgn)
    return _cache[k]


@pytest.mark.parametrize("pf", ["0", "1", "2", "3"])
def test_pipelined_passes_bit_exact(pf, monkeypatch):
    """HSFFT_PF bit 0: pf::k_firstq for pass A, bit 1: pf::k_b512 for pass B (else the
    register kernels of hsfft_pass_r8.h)"""
    monkeypatch.setenv("HSFFT_PF", pf)
    x = T.complex_input(N, 0xF00D, batch=3).reshape(3, N)
    for sgn in (1, -1):
        assert T.bits_equal(_run(x, sgn), _oracle(x, sgn, "b3")), (pf, sgn)


@pytest.mark.parametrize("nt", ["0", "2"])
def test_first_pass_2p20_nt_stores(nt, monkeypatch):
    """2^20's pass A (k_firstq<4,3,2>) with plain / non-temporal (default) output stores
    (HSFFT_PFA_NT bit 1): bit-exact, both signs"""
    monkeypatch.setenv("HSFFT_PFA_NT", nt)
    x = T.complex_input(N, 0xF00D, batch=3).reshape(3, N)
    for sgn in (1, -1):
        assert T.bits_equal(_run(x, sgn), _oracle(x, sgn, "b3")), (nt, sgn)


@pytest.mark.parametrize("q", ["1", "2", "3"])
def test_quad_load_first_pass(q, monkeypatch):
    """pf::k_firstq (64-B column loads, DPP quad swap): bit-exact, both signs, with a
    4-column-group count per row (128) that is not a multiple of 3."""
    monkeypatch.setenv("HSFFT_PF", "1")
    monkeypatch.setenv("HSFFT_PFQ", q)
    x = T.complex_input(N, 0xF00D, batch=3).reshape(3, N)
    for sgn in (1, -1):
        assert T.bits_equal(_run(x, sgn), _oracle(x, sgn, "b3")), (q, sgn)


@pytest.mark.parametrize("pfp", ["0", "1", "4"])
def test_paired_load_first_pass_2p21(pfp, monkeypatch):
    """pf::k_firstq<8,3,G=1> (2^21 = [8,8,8,8 | 8,8,8], r2c 2^22's inner c2c): 32-B paired
    column loads, L = 512 twiddles from global memory; bit-exact, both signs, odd batch."""
    monkeypatch.setenv("HSFFT_PFP", pfp)
    n = 1 << 21
    x = T.complex_input(n, 0x2121, batch=3).reshape(3, n)
    for sgn in (1, -1):
        p = hsfft.Plan(n, sgn)
        din = hsfft.DeviceBuffer.from_array(x)
        dout = hsfft.DeviceBuffer(x.nbytes)
        hsfft.exec_batched(p, din, dout, 3)
        hsfft.synchronize()
        y = dout.to_array(np.complex128).reshape(3, n)
        assert T.bits_equal(y, _oracle(x, sgn, "2p21")), (pfp, sgn)
        din.free()
        dout.free()
        p.close()


@pytest.mark.parametrize("nt", ["0", "1"])
def test_paired_load_first_pass_2p21_nt_stores(nt, monkeypatch):
    """the same pass with plain / non-temporal (default) output stores (HSFFT_PFA_NT bit 0):
    bit-exact, both signs"""
    monkeypatch.setenv("HSFFT_PFA_NT", nt)
    n = 1 << 21
    x = T.complex_input(n, 0x2121, batch=3).reshape(3, n)
    for sgn in (1, -1):
        p = hsfft.Plan(n, sgn)
        din = hsfft.DeviceBuffer.from_array(x)
        dout = hsfft.DeviceBuffer(x.nbytes)
        hsfft.exec_batched(p, din, dout, 3)
        hsfft.synchronize()
        y = dout.to_array(np.complex128).reshape(3, n)
        assert T.bits_equal(y, _oracle(x, sgn, "2p21")), sgn
        din.free()
        dout.free()
        p.close()


@pytest.mark.parametrize("n,batch,chunk_mb", [(1 << 20, 7, "32"), (4096, 33, "1"), (12600, 5, "1"), (99991, 3, "2")])
def test_host_batched_pipeline_bit_exact(n, batch, chunk_mb, monkeypatch):
    """hsfft_exec_batched_host (host rows streamed through HBM in chunks, upload / transform /
    download on three streams): bit-exact vs the oracle, odd chunk counts included."""
    monkeypatch.setenv("HSFFT_HOST_CHUNK_MB", chunk_mb)
    x = T.complex_input(n, 0xAB ^ n, batch=batch).reshape(batch, n)
    p = hsfft.Plan(n, 1)
    fb0 = hsfft.lib().hsfft_bluestein_fallbacks()
    y = hsfft.exec_batched_host(p, x)
    assert T.bits_equal(y, T.oracle_c2c(x, 1)), n
    # 99991: the pipeline's persistent launches run deferred (asynchronous, one check at the end,
    # round 6) -- none fell back, nothing is left pending
    assert hsfft.lib().hsfft_bluestein_fallbacks() == fb0
    assert hsfft.lib().hsfft_synchronize() == 0
    p.close()


@pytest.mark.parametrize("mask,xt", [("0", "3"), ("7", "0"), ("7", "3"), ("7", "7"), ("1", "3"), ("2", "3"), ("4", "3")])
@pytest.mark.parametrize("n", [99991, 65537, 131071])
def test_bluestein_row_looped_kernels(n, mask, xt, monkeypatch):
    """Bluestein with M = 2^18 (config 4's size; 65537 = 2^16+1 is the plan/exec M mismatch
    case D5, computed with its own exec-length table): the row-looped first / middle / last
    kernels (csrc/hsfft_blue_pf.h, HSFFT_BLUE_PF mask; the generic passes otherwise), both
    block orders, odd batch (a partial 8-row group), both signs, bit-exact."""
    monkeypatch.setenv("HSFFT_BLUE_XCD", "0")  # the three-launch path
    monkeypatch.setenv("HSFFT_BLUE_PF", mask)
    monkeypatch.setenv("HSFFT_BLUE_XT", xt)
    x = T.complex_input(n, 0xB1 ^ n, batch=5).reshape(5, n)
    for sgn in (1, -1):
        p = hsfft.Plan(n, sgn)
        din = hsfft.DeviceBuffer.from_array(x)
        dout = hsfft.DeviceBuffer(x.nbytes)
        hsfft.exec_batched(p, din, dout, 5)
        hsfft.synchronize()
        y = dout.to_array(np.complex128).reshape(5, n)
        assert T.bits_equal(y, _oracle(x, sgn, ("blue", n))), (n, sgn, mask, xt)
        din.free()
        dout.free()
        p.close()


@pytest.mark.parametrize("ng,batch,jitter", [("8", 1, "0"), ("8", 5, "0"), ("8", 19, "0"), ("3", 7, "0"), ("1", 2, "0"),
                                             ("8", 19, "3"), ("3", 7, "5")])
@pytest.mark.parametrize("n", [99991, 65537, 131071])
def test_bluestein_persistent_launch(n, ng, batch, jitter, monkeypatch):
    """Bluestein M = 2^18 as one persistent launch (csrc/hsfft_blue_xcd.h: groups of 64
    workgroups carry a row through the three passes, intermediates handed over in-launch):
    fewer rows than groups, ragged last round, both signs, and under uneven load (HSFFT_BX_JITTER:
    pseudo-random per-phase delays scramble the hand-off order) -- bit-exact vs the oracle and
    vs the three-launch path; no launch fell back."""
    monkeypatch.setenv("HSFFT_BLUE_XCD", ng)
    monkeypatch.setenv("HSFFT_BX_JITTER", jitter)
    fb0 = hsfft.lib().hsfft_bluestein_fallbacks()
    x = T.complex_input(n, 0xB7 ^ n ^ batch, batch=batch).reshape(batch, n)
    for sgn in (1, -1):
        p = hsfft.Plan(n, sgn)
        din = hsfft.DeviceBuffer.from_array(x)
        dout = hsfft.DeviceBuffer(x.nbytes)
        hsfft.exec_batched(p, din, dout, batch)
        hsfft.synchronize()
        y = dout.to_array(np.complex128).reshape(batch, n)
        assert T.bits_equal(y, _oracle(x, sgn, ("bxcd", n, batch))), (n, sgn, ng, batch)
        monkeypatch.setenv("HSFFT_BLUE_XCD", "0")
        dout.fill_zero()
        hsfft.exec_batched(p, din, dout, batch)
        hsfft.synchronize()
        assert T.bits_equal(dout.to_array(np.complex128).reshape(batch, n), y)
        monkeypatch.setenv("HSFFT_BLUE_XCD", ng)
        din.free()
        dout.free()
        p.close()
    assert hsfft.lib().hsfft_bluestein_fallbacks() == fb0


@pytest.mark.parametrize("ng,batch,jitter", [("8", 19, "0"), ("3", 7, "5"), ("8", 1, "0")])
@pytest.mark.parametrize("n", [99991, 65537, 131071])
def test_bluestein_persistent_unconditional_loads(n, ng, batch, jitter, monkeypatch):
    """k_bxcd's loads (round 5): P1's row / chirp loads and P3's chirp loads issued
    unconditionally at clamped indices, the padding and the n < N store condition applied to
    the values -- bit-exact vs the oracle at lengths whose last tile is partly padding, both
    signs, 1 / 3 / 8 groups, uneven load"""
    monkeypatch.setenv("HSFFT_BLUE_XCD", ng)
    monkeypatch.setenv("HSFFT_BX_JITTER", jitter)
    fb0 = hsfft.lib().hsfft_bluestein_fallbacks()
    x = T.complex_input(n, 0xB8 ^ n ^ batch, batch=batch).reshape(batch, n)
    for sgn in (1, -1):
        p = hsfft.Plan(n, sgn)
        din = hsfft.DeviceBuffer.from_array(x)
        dout = hsfft.DeviceBuffer(x.nbytes)
        hsfft.exec_batched(p, din, dout, batch)
        hsfft.synchronize()
        y = dout.to_array(np.complex128).reshape(batch, n)
        assert T.bits_equal(y, _oracle(x, sgn, ("bxul", n, batch))), (n, sgn, ng, batch)
        din.free()
        dout.free()
        p.close()
    assert hsfft.lib().hsfft_bluestein_fallbacks() == fb0


@pytest.mark.parametrize("mode", ["refused", "sync", "census_sync", "unchecked_async"])
def test_bluestein_persistent_launch_contract(mode, monkeypatch):
    """The persistent Bluestein launch needs every workgroup of a group resident at once.
    refused: 9 groups = 576 workgroups of which only 512 (two per CU) can be resident, so the
    host's occupancy check refuses the grid and the rows run on the three-launch path at once --
    results bit-exact, one fallback counted per call, no ~1 s wait.  sync: HSFFT_BX_SYNC=1 (the
    synchronous form with the automatic re-run) -- bit-exact, no fallback.
    Round 6, the in-kernel arrival census, with the host check skipped
    (HSFFT_BX_UNCHECKED=1) so the oversized grid is really launched:
      census_sync: the 9 groups' workgroups interleaved (HSFFT_BX_MAP=0: group = block % 9), so
        every group is partly resident and none can finish; the synchronous call's census gives
        up after ~2 ms without a new arrival and the rows re-run on the three-launch path --
        bit-exact, one fallback, well under the ~1.3 s hand-off bound;
      unchecked_async: groups of 64 consecutive blocks (the default map): groups 0-7 are
        resident and complete, group 8 is dispatched into the slots they free and its census
        completes then -- an oversized grid is slower, not failed: bit-exact, no fallback, no
        pending error."""
    import time
    n, batch = 99991, 11
    monkeypatch.setenv("HSFFT_BLUE_XCD", "8" if mode == "sync" else "9")
    if mode in ("sync", "census_sync"):
        monkeypatch.setenv("HSFFT_BX_SYNC", "1")
    if mode in ("census_sync", "unchecked_async"):
        monkeypatch.setenv("HSFFT_BX_UNCHECKED", "1")
    if mode == "census_sync":
        monkeypatch.setenv("HSFFT_BX_MAP", "0")
    x = T.complex_input(n, 0xC0C0, batch=batch).reshape(batch, n)
    ref = _oracle(x, 1, ("coop", n, batch))
    p = hsfft.Plan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(x.nbytes)
    for it in range(2):
        fb0 = hsfft.lib().hsfft_bluestein_fallbacks()
        dout.fill_zero()
        t0 = time.perf_counter()
        hsfft.exec_batched(p, din, dout, batch)
        hsfft.synchronize()
        dt = time.perf_counter() - t0
        assert T.bits_equal(dout.to_array(np.complex128).reshape(batch, n), ref), (mode, it)
        assert hsfft.lib().hsfft_bluestein_fallbacks() == fb0 + (1 if mode in ("refused", "census_sync") else 0), mode
        assert dt < 0.5, f"{mode}: {dt:.3f} s for {batch} rows (a refused launch must not wait)"
    din.free()
    dout.free()
    p.close()


def test_bluestein_async_timeout_reported_once(monkeypatch):
    """The asynchronous error contract of the persistent launch (include/hsfft_gpu.h), with its
    in-launch waits forced to time out (HSFFT_BX_TLIMIT=1 tick of 10 ns, HSFFT_BX_JITTER=5
    uneven arrivals):
      1. hsfft_exec_batched (asynchronous) returns 0 and leaves the error pending;
      2. calls on OTHER plans that shrink / regrow the scratch pool and build device state
         (hsfft_release_scratch, an r2c of 2^22, a drop-in fft_exec of 1024) succeed, are
         bit-exact and do not consume the error;
      3. the next hsfft_synchronize() returns HSFFT_ERR_DEVICE, the one after it 0 (once);
      4. the same forced timeout in a synchronous call -- HSFFT_BX_SYNC=1, and the drop-in
         fft_exec on host buffers -- re-runs the rows on the three-launch path: bit-exact, one
         fallback counted per call, and nothing left pending."""
    n, batch = 99991, 8
    x = T.complex_input(n, 0x7173, batch=batch).reshape(batch, n)
    ref = _oracle(x, 1, ("tlimit", n, batch))
    p = hsfft.Plan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(x.nbytes)
    L = hsfft.lib()
    assert L.hsfft_synchronize() == 0
    monkeypatch.setenv("HSFFT_BLUE_XCD", "8")
    monkeypatch.setenv("HSFFT_BX_TLIMIT", "1")
    monkeypatch.setenv("HSFFT_BX_JITTER", "5")
    fb0 = L.hsfft_bluestein_fallbacks()
    assert L.hsfft_exec_batched(p.ptr, hsfft.VP(din.ptr), hsfft.VP(dout.ptr), batch) == 0
    monkeypatch.delenv("HSFFT_BX_TLIMIT")
    monkeypatch.delenv("HSFFT_BX_JITTER")
    assert L.hsfft_bluestein_fallbacks() == fb0, "an asynchronous call does not re-run rows"
    # 2. other plans' calls: scratch released and regrown, device states built
    assert L.hsfft_release_scratch() == 0
    nr = 1 << 22
    xr = T.real_input(nr, 0x52, batch=1)
    rp = hsfft.RealPlan(nr, 1)
    dxr = hsfft.DeviceBuffer.from_array(xr)
    dyr = hsfft.DeviceBuffer(nr * 16)
    assert L.hsfft_r2c_batched(rp.ptr, hsfft.VP(dxr.ptr), hsfft.VP(dyr.ptr), 1) == 0
    small = hsfft.Plan(1024, -1)
    xs = T.complex_input(1024, 0x53)
    ys = small.exec(xs)
    assert T.bits_equal(ys, T.oracle_c2c(xs, -1))
    # 3. reported exactly once, by hsfft_synchronize
    assert L.hsfft_synchronize() == hsfft.HSFFT_ERR_DEVICE
    assert b"timed out" in L.hsfft_last_error()
    assert L.hsfft_synchronize() == 0
    assert T.bits_equal(dyr.to_array(np.complex128), T.oracle_r2c(xr, 1))
    # 4. synchronous forms re-run the rows
    monkeypatch.setenv("HSFFT_BX_TLIMIT", "1")
    monkeypatch.setenv("HSFFT_BX_JITTER", "5")
    monkeypatch.setenv("HSFFT_BX_SYNC", "1")
    dout.fill_zero()
    fb1 = L.hsfft_bluestein_fallbacks()
    assert L.hsfft_exec_batched(p.ptr, hsfft.VP(din.ptr), hsfft.VP(dout.ptr), batch) == 0
    assert L.hsfft_synchronize() == 0
    assert L.hsfft_bluestein_fallbacks() == fb1 + 1
    assert T.bits_equal(dout.to_array(np.complex128).reshape(batch, n), ref)
    monkeypatch.delenv("HSFFT_BX_SYNC")
    y1 = p.exec(x[3])  # the drop-in fft_exec on host buffers is synchronous by itself
    assert L.hsfft_bluestein_fallbacks() == fb1 + 2
    assert T.bits_equal(y1, ref[3])
    assert L.hsfft_synchronize() == 0
    # 5. the host pipeline keeps its launches asynchronous and reads its own DEFERRED error word
    # once at the end (round 6): the timed-out batch re-runs on the three-launch path
    # -- bit-exact, one fallback, nothing left for hsfft_synchronize()
    monkeypatch.setenv("HSFFT_HOST_CHUNK_MB", "4")  # 3 chunks of 2 rows + 2
    yh = hsfft.exec_batched_host(p, x)
    assert L.hsfft_bluestein_fallbacks() == fb1 + 3
    assert T.bits_equal(yh, ref)
    assert L.hsfft_synchronize() == 0
    for d in (din, dout, dxr, dyr):
        d.free()
    p.close()
    rp.close()
    small.close()


def test_bluestein_persistent_beside_concurrent_small_calls(monkeypatch):
    """the persistent grid fills the chip (2 workgroups per CU x 256 CUs), and
    the concurrent small fft_exec path launches one-workgroup kernels on per-thread streams
    outside the device lock, so a small kernel can hold a slot the persistent grid needs.  One
    thread runs asynchronous 99991-point batches (the persistent launch) while another issues
    drop-in fft_exec calls of 1024 points throughout: no launch fell back, no error is pending,
    every Bluestein output word equals the same rows run alone, sampled rows equal the oracle,
    and every small call is bit-exact."""
    import threading
    monkeypatch.setenv("HSFFT_BLUE_XCD", "8")
    n, batch, iters = 99991, 64, 6
    L = hsfft.lib()
    x = T.complex_input(n, 0x5EED, batch=batch).reshape(batch, n)
    p = hsfft.Plan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    d_alone = hsfft.DeviceBuffer(x.nbytes)
    d_conc = hsfft.DeviceBuffer(x.nbytes)
    assert L.hsfft_synchronize() == 0
    hsfft.exec_batched(p, din, d_alone, batch)
    assert L.hsfft_synchronize() == 0
    small = hsfft.Plan(1024, -1)
    xs = [T.complex_input(1024, 0x600 + k) for k in range(4)]
    refs = [T.oracle_c2c(v, -1) for v in xs]
    stop = threading.Event()
    errors, calls = [], [0]

    def small_worker():
        try:
            L.hsfft_set_device(0)
            k = 0
            while not stop.is_set():
                y = small.exec(xs[k % 4])
                if not T.bits_equal(y, refs[k % 4]):
                    errors.append(("small", k))
                k += 1
            calls[0] = k
        except Exception as e:  # pragma: no cover
            errors.append(("exception", repr(e)))

    fb0 = L.hsfft_bluestein_fallbacks()
    th = threading.Thread(target=small_worker)
    th.start()
    try:
        for it in range(iters):
            d_conc.fill_zero()
            assert L.hsfft_exec_batched(p.ptr, hsfft.VP(din.ptr), hsfft.VP(d_conc.ptr), batch) == 0
            assert L.hsfft_synchronize() == 0, (it, L.hsfft_last_error())
            diff = hsfft.count_diff_words(d_alone, d_conc, x.nbytes)
            assert diff == 0, (it, diff)
    finally:
        stop.set()
        th.join(timeout=120)
    assert not th.is_alive()
    assert not errors, errors[:5]
    assert calls[0] > 0
    assert L.hsfft_bluestein_fallbacks() == fb0
    y = d_alone.to_array(np.complex128).reshape(batch, n)
    rows = [0, 37, batch - 1]
    assert T.bits_equal(y[rows], _oracle(x[rows], 1, ("conc", n, 3)))
    for d in (din, d_alone, d_conc):
        d.free()
    p.close()
    small.close()


@pytest.mark.parametrize("jitter", ["0", "2"])
def test_bluestein_persistent_full_size_every_word(jitter, monkeypatch):
    """BASELINE config 4 at full size (99991 x 8192) through the persistent launch, compared on
    EVERY output word with the three-launch path (no in-launch hand-off), plus sampled rows vs
    the oracle.  jitter 2 runs it under uneven load (random per-phase delays of 0-2 units).
    The persistent launch reuses each image every two rows, so its consumers read lines their
    CU read before (L1-warm), as MI355X_MICROARCH.md asks hand-off tests to do."""
    n, batch = 99991, 8192
    monkeypatch.setenv("HSFFT_BX_JITTER", jitter)
    p = hsfft.Plan(n, 1)
    din = hsfft.DeviceBuffer(batch * n * 16)
    d1 = hsfft.DeviceBuffer(batch * n * 16)
    d2 = hsfft.DeviceBuffer(batch * n * 16)
    hsfft.fill_complex(din, batch * n, T.SEEDS[4])
    fb0 = hsfft.lib().hsfft_bluestein_fallbacks()
    monkeypatch.setenv("HSFFT_BLUE_XCD", "8")
    hsfft.exec_batched(p, din, d1, batch)
    hsfft.synchronize()
    assert hsfft.lib().hsfft_bluestein_fallbacks() == fb0, "the persistent launch fell back"
    monkeypatch.setenv("HSFFT_BLUE_XCD", "0")
    hsfft.exec_batched(p, din, d2, batch)
    hsfft.synchronize()
    rows = 256  # compared in chunks of 256 rows (410 MB per buffer)
    bad = 0
    for r0 in range(0, batch, rows):
        off = r0 * n * 16
        a = d1.to_array(np.complex128, rows * n, off)
        b = d2.to_array(np.complex128, rows * n, off)
        bad += int((a.view(np.uint64) != b.view(np.uint64)).sum())
    assert bad == 0, f"{bad} 8-byte words differ between the persistent and the three-launch path"
    for row in (0, 4097, batch - 1):
        x = T.complex_input(n, T.SEEDS[4], batch=1, row0=row)
        y = d1.to_array(np.complex128, n, row * n * 16)
        assert T.bits_equal(y, _oracle(x, 1, ("c4row", row))), row
    for d in (din, d1, d2):
        d.free()
    p.close()


@pytest.mark.parametrize("fuse", ["0", "1"])
@pytest.mark.parametrize("n,batch", [(8, 3), (1000, 5), (1 << 16, 4), (1 << 19, 3), (1 << 22, 2), (2 * 99991, 2)])
def test_r2c_compact_bit_exact(n, batch, fuse, monkeypatch):
    """hsfft_r2c_batched_compact: bins 0..N/2 per row, bit-identical to the reference-layout
    output's first N/2+1 bins (and so to the oracle); split fused into the last pass or not"""
    monkeypatch.setenv("HSFFT_R2C_FUSE", fuse)
    x = T.real_input(n, 0xC0 ^ n, batch=batch).reshape(batch, n)
    rp = hsfft.RealPlan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(batch * (n // 2 + 1) * 16)
    hsfft.r2c_batched_compact(rp, din, dout, batch)
    y = dout.to_array(np.complex128).reshape(batch, n // 2 + 1)
    ref = T.oracle_r2c(x, 1).reshape(batch, n)
    assert T.bits_equal(y, np.ascontiguousarray(ref[:, :n // 2 + 1]))
