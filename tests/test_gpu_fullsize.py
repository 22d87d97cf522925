"""Every-word parity of the default schedules at BASELINE's full per-GPU sizes.

Sampled rows against the oracle cannot see a boundary error of a walking kernel in a row that
is not sampled (k_firstq walks column tiles, k_b512 row groups, k_row2 grid-strides rows and
prefetches the next row's first group, k_r2c_walk1 carries one entry across tiles in eight
rotation classes).  So each config's default schedule is compared on EVERY 8-byte output word
with an independent in-library schedule of the same transform (different kernels, different
walk / tile structure, itself bit-exact vs the oracle in test_gpu_parity.py), on the GPU
(hsfft_count_diff_words), plus sampled rows vs the oracle:

* c2  4096 x 2^20 c2c: pf::k_firstq + pf::k_b512  vs  HSFFT_PF=0 (r8::k_pass both passes);
* c3  65536 x 12600 c2c: mr::k_row2 (one pass)  vs  HSFFT_MR_ROW=0 (two mr::k_pass passes);
* c5  512 x 2^22 r2c (the bench's call size): pf::k_r2c_walk1 (default since round 4)  vs
  HSFFT_R2C_WALK=0 (pf::k_r2c_fused, one tile pair per workgroup).

Reference: highSpeedFFT.c:1920-1942 (fft_exec), real.c:78-136 (fft_r2c_exec).
Tolerance: bit-exact (0 differing words).
"""
import numpy as np
import pytest

import hsfft_testlib as T

import hsfft

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if hsfft.device_count() < 1:
        pytest.skip("no GPU")
    hsfft.lib().hsfft_set_device(0)
    hsfft.lib().hsfft_release_scratch()  # earlier modules' pools: these tests need ~200 GiB
    yield
    hsfft.synchronize()
    hsfft.lib().hsfft_release_scratch()


def _comparator_self_check(a, b, nbytes):
    """the GPU comparator itself: equal buffers give 0, one flipped word gives 1"""
    assert hsfft.count_diff_words(a, a, nbytes) == 0
    off = (nbytes // 2) // 8 * 8
    keep = b.to_array(np.uint64, 1, off)
    hsfft.check(hsfft.lib().hsfft_memset(hsfft.VP(b.ptr + off), 0x5A, 8), "memset")
    assert hsfft.count_diff_words(a, b, nbytes) == 1
    hsfft.check(hsfft.lib().hsfft_memcpy_h2d(hsfft.VP(b.ptr + off), keep.ctypes.data_as(hsfft.VP), 8), "h2d")


def _c2c_every_word(n, batch, seed, env_alt, rows, monkeypatch, sgn=1):
    p = hsfft.Plan(n, sgn)
    nbytes = batch * n * 16
    din = hsfft.DeviceBuffer(nbytes)
    d1 = hsfft.DeviceBuffer(nbytes)
    d2 = hsfft.DeviceBuffer(nbytes)
    hsfft.fill_complex(din, batch * n, seed)
    d1.fill_zero()
    d2.fill_zero()
    hsfft.exec_batched(p, din, d1, batch)  # default schedule
    hsfft.synchronize()
    for k, v in env_alt.items():
        monkeypatch.setenv(k, v)
    hsfft.exec_batched(p, din, d2, batch)  # the independent schedule
    hsfft.synchronize()
    for k in env_alt:
        monkeypatch.delenv(k)
    bad = hsfft.count_diff_words(d1, d2, nbytes)
    assert bad == 0, f"N={n} x {batch}: {bad} 8-byte words differ between the default schedule and {env_alt}"
    _comparator_self_check(d1, d2, nbytes)
    for row in rows:
        y = d1.to_array(np.complex128, n, row * n * 16)
        x = T.complex_input(n, seed, batch=1, row0=row)
        assert T.bits_equal(y, T.oracle_c2c(x.reshape(1, n), sgn)[0]), row
    for d in (din, d1, d2):
        d.free()
    p.close()


def test_config2_every_word(monkeypatch):
    """4096 x 2^20 (64 GiB each way): k_firstq + k_b512 vs the register passes, every word"""
    _c2c_every_word(1 << 20, 4096, T.SEEDS[2], {"HSFFT_PF": "0"}, (0, 2049, 4095), monkeypatch)


def test_config3_every_word(monkeypatch):
    """65536 x 12600: the row kernel vs the two mixed-radix passes, every word"""
    _c2c_every_word(12600, 65536, T.SEEDS[3], {"HSFFT_MR_ROW": "0"}, (0, 257, 65535), monkeypatch)


def test_config5_every_word(monkeypatch):
    """512 x 2^22 reals (the bench's r2c call size): the default split walk vs one tile pair per
    workgroup, every word of the mirrored N-bin output; sampled rows vs the oracle"""
    n, batch = 1 << 22, 512
    rp = hsfft.RealPlan(n, 1)
    din = hsfft.DeviceBuffer(batch * n * 8)
    nbytes = batch * n * 16
    d1 = hsfft.DeviceBuffer(nbytes)
    d2 = hsfft.DeviceBuffer(nbytes)
    hsfft.fill_real(din, batch * n, T.SEEDS[5])
    hsfft.fill_complex(d1, batch * n, 1)  # stale data: every bin must be written
    hsfft.fill_complex(d2, batch * n, 2)
    hsfft.r2c_batched(rp, din, d1, batch)
    hsfft.synchronize()
    for walk, name in (("0", "k_r2c_fused"),):
        monkeypatch.setenv("HSFFT_R2C_WALK", walk)
        hsfft.fill_complex(d2, batch * n, 2)
        hsfft.r2c_batched(rp, din, d2, batch)
        hsfft.synchronize()
        monkeypatch.delenv("HSFFT_R2C_WALK")
        bad = hsfft.count_diff_words(d1, d2, nbytes)
        assert bad == 0, f"{bad} 8-byte words differ between the default split walk and {name}"
    _comparator_self_check(d1, d2, nbytes)
    for row in (0, 257, batch - 1):
        y = d1.to_array(np.complex128, n, row * n * 16)
        x = T.real_input(n, T.SEEDS[5], batch=1, row0=row)
        assert T.bits_equal(y, T.oracle_r2c(x.reshape(1, n), 1)[0]), row
    for d in (din, d1, d2):
        d.free()
    rp.close()
