"""GPU parity of the 2^20 hot-path kernel families (BASELINE config 2) against the oracle:

* pf::k_firstq / pf::k_first / pf::k_b512 (csrc/hsfft_pass_pf.h): the two-launch passes
  (64-B quad-load first pass, its 32-B predecessor, the row-looped later pass);
* fz::k_fused (csrc/hsfft_fused.h): both passes in one persistent launch with the
  intermediate handed over inside the launch (HSFFT_FUSED=1).

Tolerance: bit-exact (0 ulp) against the oracle (the CPU restatement pinned to the reference)
and against the two-launch path.  Batch sizes cover a partial last row group, a single row
(R falls back to 1), every rows-per-group setting and lags larger than the group count.
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


@pytest.mark.parametrize("pf,pfq", [("0", "4"), ("1", "4"), ("2", "4"), ("3", "4"), ("3", "0")])
def test_pipelined_passes_bit_exact(pf, pfq, monkeypatch):
    monkeypatch.setenv("HSFFT_PF", pf)
    monkeypatch.setenv("HSFFT_PFQ", pfq)
    x = T.complex_input(N, 0xF00D, batch=3).reshape(3, N)
    for sgn in (1, -1):
        assert T.bits_equal(_run(x, sgn), _oracle(x, sgn, "b3")), (pf, sgn)


@pytest.mark.parametrize("g,t", [(1, 8), (2, 2), (2, 8), (4, 4)])
def test_pipelined_first_pass_tiles(g, t, monkeypatch):
    monkeypatch.setenv("HSFFT_PF", "1")
    monkeypatch.setenv("HSFFT_PFQ", "0")
    monkeypatch.setenv("HSFFT_PFG", str(g))
    monkeypatch.setenv("HSFFT_PFT", str(t))
    x = T.complex_input(N, 0xF00D, batch=3).reshape(3, N)
    assert T.bits_equal(_run(x, 1), _oracle(x, 1, "b3"))


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


@pytest.mark.parametrize("batch,r,lag", [(1, 2, 2), (2, 2, 2), (6, 2, 2), (8, 4, 1), (5, 1, 3), (6, 2, 9)])
def test_fused_bit_exact(batch, r, lag, monkeypatch):
    monkeypatch.setenv("HSFFT_FUSED", "1")
    monkeypatch.setenv("HSFFT_FZ_R", str(r))
    monkeypatch.setenv("HSFFT_FZ_LAG", str(lag))
    x = T.complex_input(N, 0xF00D ^ batch, batch=batch).reshape(batch, N)
    for sgn in (1, -1):
        y = _run(x, sgn)
        ref = _oracle(x, sgn, ("f", batch))
        assert T.bits_equal(y, ref), (batch, r, lag, sgn, T.mismatches(y, ref))


@pytest.mark.parametrize("mode", ["1"])
def test_fused_large_batch_vs_two_launch(mode, monkeypatch):
    """64 rows (16 GiB of pass traffic): the fused launch equals the two-launch path bit for
    bit on every row and the oracle on sampled rows; no dependency wait timed out."""
    batch = 64
    p = hsfft.Plan(N, 1)
    din = hsfft.DeviceBuffer(batch * N * 16)
    d2 = hsfft.DeviceBuffer(batch * N * 16)
    d1 = hsfft.DeviceBuffer(batch * N * 16)
    hsfft.fill_complex(din, batch * N, T.SEEDS[2])
    monkeypatch.setenv("HSFFT_FUSED", "0")
    hsfft.exec_batched(p, din, d2, batch)
    hsfft.synchronize()
    monkeypatch.setenv("HSFFT_FUSED", mode)
    d1.fill_zero()
    hsfft.exec_batched(p, din, d1, batch)
    hsfft.synchronize()
    a = d1.to_array(np.complex128)
    b = d2.to_array(np.complex128)
    assert T.bits_equal(a, b)
    for row in (0, 37, batch - 1):
        x = T.complex_input(N, T.SEEDS[2], batch=1, row0=row)
        assert T.bits_equal(a[row * N:(row + 1) * N], T.oracle_c2c(x, 1)), row
    for d in (din, d1, d2):
        d.free()


@pytest.mark.parametrize("n,batch,chunk_mb", [(1 << 20, 7, "32"), (4096, 33, "1"), (12600, 5, "1"), (99991, 3, "2")])
def test_host_batched_pipeline_bit_exact(n, batch, chunk_mb, monkeypatch):
    """hsfft_exec_batched_host (host rows streamed through HBM in chunks, upload / transform /
    download on three streams): bit-exact vs the oracle, odd chunk counts included."""
    monkeypatch.setenv("HSFFT_HOST_CHUNK_MB", chunk_mb)
    x = T.complex_input(n, 0xAB ^ n, batch=batch).reshape(batch, n)
    p = hsfft.Plan(n, 1)
    y = hsfft.exec_batched_host(p, x)
    assert T.bits_equal(y, T.oracle_c2c(x, 1)), n
    p.close()


@pytest.mark.parametrize("mask,t,pref", [("0", "4", "0"), ("3", "1", "0"), ("3", "2", "0"), ("3", "4", "0"), ("3", "8", "0"),
                                         ("7", "8", "1"), ("1", "4", "0"), ("2", "4", "0")])
@pytest.mark.parametrize("n", [99991, 65537, 131071])
def test_bluestein_row_looped_kernels(n, mask, t, pref, monkeypatch):
    """Bluestein with M = 2^18 (config 4's size; 65537 = 2^16+1 is the plan/exec M mismatch
    case D5, computed with its own exec-length table): the row-looped middle / last kernels
    (csrc/hsfft_blue_pf.h) for every tile-row count, odd batch, both signs, bit-exact."""
    monkeypatch.setenv("HSFFT_BLUE_XCD", "0")  # the three-launch path
    monkeypatch.setenv("HSFFT_BLUE_PF", mask)
    monkeypatch.setenv("HSFFT_BLUE_T", t)
    monkeypatch.setenv("HSFFT_BLUE_PREF", pref)
    monkeypatch.setenv("HSFFT_BLUE_XT", "0" if t == "2" else "3")  # both block orders
    x = T.complex_input(n, 0xB1 ^ n, batch=5).reshape(5, n)
    for sgn in (1, -1):
        p = hsfft.Plan(n, sgn)
        din = hsfft.DeviceBuffer.from_array(x)
        dout = hsfft.DeviceBuffer(x.nbytes)
        hsfft.exec_batched(p, din, dout, 5)
        hsfft.synchronize()
        y = dout.to_array(np.complex128).reshape(5, n)
        assert T.bits_equal(y, _oracle(x, sgn, ("blue", n))), (n, sgn, mask, t)
        din.free()
        dout.free()
        p.close()


@pytest.mark.parametrize("ng,batch", [("8", 1), ("8", 5), ("8", 19), ("3", 7), ("1", 2)])
@pytest.mark.parametrize("n", [99991, 65537, 131071])
def test_bluestein_persistent_launch(n, ng, batch, monkeypatch):
    """Bluestein M = 2^18 as one persistent launch (csrc/hsfft_blue_xcd.h: groups of 64
    workgroups carry a row through the three passes, intermediates handed over in-launch):
    fewer rows than groups, ragged last round, both signs -- bit-exact vs the oracle and vs
    the three-launch path."""
    monkeypatch.setenv("HSFFT_BLUE_XCD", ng)
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
