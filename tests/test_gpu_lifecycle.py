"""hsfft_finalize() in the middle of a process (round 5; include/hsfft_gpu.h): it releases every
device object the library holds -- streams, events, scratch pools, per-plan device states, the
persistent Bluestein launch's counter block and error words -- and the library stays usable:
the same plans and caller buffers run again, rebuilding what they need, bit-exact vs the oracle.
Covers the four hot schedules (2^20 two-pass, the 12600 row kernel, the persistent Bluestein
launch, the chunked r2c walk) and the drop-in fft_exec on host buffers."""
import numpy as np
import pytest

import hsfft_testlib as T

import hsfft

pytestmark = pytest.mark.gpu


def _c2c_case(n, batch, seed):
    x = T.complex_input(n, seed, batch=batch).reshape(batch, n)
    p = hsfft.Plan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(x.nbytes)

    def run():
        dout.fill_zero()
        hsfft.exec_batched(p, din, dout, batch)
        hsfft.synchronize()
        return dout.to_array(np.complex128).reshape(batch, n)

    return run, T.oracle_c2c(x, 1), (p, din, dout)


def _r2c_case(n, batch, seed):
    x = T.real_input(n, seed, batch=batch).reshape(batch, n)
    p = hsfft.RealPlan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(batch * n * 16)

    def run():
        dout.fill_zero()
        hsfft.r2c_batched(p, din, dout, batch)
        hsfft.synchronize()
        return dout.to_array(np.complex128).reshape(batch, n)

    return run, T.oracle_r2c(x, 1), (p, din, dout)


def test_finalize_then_reuse():
    if hsfft.device_count() < 1:
        pytest.skip("no GPU")
    hsfft.lib().hsfft_set_device(0)
    fb0 = hsfft.lib().hsfft_bluestein_fallbacks()
    cases = {
        "2^20": _c2c_case(1 << 20, 2, 0x51),
        "12600": _c2c_case(12600, 3, 0x52),
        "99991": _c2c_case(99991, 2, 0x53),
        "r2c 2^22": _r2c_case(1 << 22, 1, 0x54),
    }
    small = hsfft.Plan(1024, 1)
    xs = T.complex_input(1024, 0x55, batch=1)
    ref_small = T.oracle_c2c(xs.reshape(1, 1024), 1).reshape(1024)
    for rnd in range(2):
        for name, (run, ref, _) in cases.items():
            assert T.bits_equal(run(), ref), (name, rnd)
        assert T.bits_equal(small.exec(xs), ref_small), ("fft_exec", rnd)
        assert hsfft.finalize() == 0, hsfft.lib().hsfft_last_error()
    assert hsfft.finalize() == 0  # nothing left to release: still fine
    # the persistent Bluestein launch ran both times (its counter block was re-created)
    assert hsfft.lib().hsfft_bluestein_fallbacks() == fb0
    for _, _, objs in cases.values():
        p, din, dout = objs
        din.free()
        dout.free()
        p.close()
    small.close()
