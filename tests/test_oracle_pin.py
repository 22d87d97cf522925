"""Live pin of the oracle against the unmodified reference build (oracle/_ref/libhsref.so).
Skipped where the reference was not built (the GPU box relies on test_oracle_golden)."""
import ctypes

import numpy as np
import pytest

import hsfft_testlib as T

ref = T.reference()
pytestmark = pytest.mark.skipif(ref is None, reason="reference build oracle/_ref absent")

ASIS_SIZES = [3, 4, 5, 7, 8, 9, 12, 15, 16, 20, 25, 27, 32, 36, 45, 49, 60, 64, 100, 125, 243,
              343, 256, 512, 4096, 12600, 11, 22, 121, 17, 92, 87, 31, 185, 41, 43, 47, 106, 88,
              19, 97, 1021, 5003]


@pytest.mark.parametrize("n", ASIS_SIZES)
def test_oracle_equals_reference_asis(n):
    rng = np.random.default_rng(n)
    for sgn in (1, -1):
        x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
        y = np.zeros(n, dtype=np.complex128)
        p = ref.fft_init(n, sgn)
        ref.fft_exec(p, T.ptr(x), T.ptr(y))
        ref.free_fft(p)
        assert T.bits_equal(T.oracle_c2c(x, sgn, T.ORC_LEAF2_ASIS), y)


def test_factors_and_dividebyN_exhaustive():
    lib = T.oracle()
    a = np.zeros(64, dtype=np.int32)
    b = np.zeros(64, dtype=np.int32)
    for n in range(1, 1 << 16):
        assert lib.orc_dividebyN(n) == ref.dividebyN(n), n
        ka = lib.orc_factors(n, T.ptr(a))
        kb = ref.factors(n, T.ptr(b))
        assert ka == kb and np.array_equal(a[:ka], b[:kb]), n


def test_twiddle_bytes_equal_reference_plan():
    for n in [12, 36, 1024, 12600, 99991, 1 << 16]:
        for sgn in (1, -1):
            p = ref.fft_init(n, sgn)
            hdr = (ctypes.c_int * 68).from_address(p)
            lf = hdr[66]
            m = int(np.prod([hdr[2 + i] for i in range(lf)]))
            rtw = np.frombuffer(bytes((ctypes.c_double * (2 * (m - 1))).from_address(p + 272)), dtype=np.complex128)
            ref.free_fft(p)
            tw, _, _, om = T.oracle_plan_twiddles(n, sgn, 0)
            assert om == m and T.bits_equal(tw, rtw)
