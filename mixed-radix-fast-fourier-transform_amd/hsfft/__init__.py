"""hsfft -- Python (ctypes) binding of libhsfft.so, the MI355X drop-in for highSpeedFFT.

The product is the C-ABI library lib/libhsfft.so (include/highspeedFFT.h, include/real.h,
include/hsfft_gpu.h).  This module only binds it for tests and bench.py; it contains no
compute.  Loading fails loudly if the library was not built (run __graft_entry__.build()
or `make -C mixed-radix-fast-fourier-transform_amd`).
"""
import ctypes
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("HSFFT_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libhsfft.so")

VP = ctypes.c_void_p
CI = ctypes.c_int

# public symbols of include/*.h with their ctypes signatures (tests check every one exists)
SIGNATURES = {
    # highspeedFFT.h
    "fft_init": (VP, [CI, CI]),
    "fft_exec": (None, [VP, VP, VP]),
    "divideby": (CI, [CI, CI]),
    "dividebyN": (CI, [CI]),
    "factors": (CI, [CI, VP]),
    "twiddle": (None, [VP, CI, CI]),
    "longvectorN": (None, [VP, CI, VP, CI]),
    "free_fft": (None, [VP]),
    # real.h
    "fft_real_init": (VP, [CI, CI]),
    "fft_r2c_exec": (None, [VP, VP, VP]),
    "fft_c2r_exec": (None, [VP, VP, VP]),
    "free_real_fft": (None, [VP]),
    "fft_convolve": (CI, [ctypes.c_char_p, ctypes.c_char_p, VP, CI, VP, CI, VP]),
    "next_power_of_two": (CI, [CI]),
    "find_optimal_fft_length": (CI, [CI, ctypes.c_char_p, CI, CI]),
    # hsfft_gpu.h
    "hsfft_device_count": (CI, []),
    "hsfft_set_device": (CI, [CI]),
    "hsfft_get_device": (CI, []),
    "hsfft_malloc": (VP, [ctypes.c_size_t]),
    "hsfft_free": (CI, [VP]),
    "hsfft_memcpy_h2d": (CI, [VP, VP, ctypes.c_size_t]),
    "hsfft_memcpy_d2h": (CI, [VP, VP, ctypes.c_size_t]),
    "hsfft_memset": (CI, [VP, CI, ctypes.c_size_t]),
    "hsfft_synchronize": (CI, []),
    "hsfft_release_scratch": (CI, []),
    "hsfft_finalize": (CI, []),
    "hsfft_get_stream": (VP, []),
    "hsfft_last_error": (ctypes.c_char_p, []),
    "hsfft_set_twiddle_mode": (CI, [CI]),
    "hsfft_get_twiddle_mode": (CI, []),
    "hsfft_plan_refresh": (CI, [VP]),
    "hsfft_plan_num_passes": (CI, [VP]),
    "hsfft_digit_reverse_map": (CI, [VP, VP]),
    "hsfft_exec_batched": (CI, [VP, VP, VP, CI]),
    "hsfft_exec_batched_host": (CI, [VP, VP, VP, CI]),
    "hsfft_r2c_batched": (CI, [VP, VP, VP, CI]),
    "hsfft_r2c_batched_compact": (CI, [VP, VP, VP, CI]),
    "hsfft_c2r_batched": (CI, [VP, VP, VP, CI]),
    "hsfft_convolve_batched": (CI, [ctypes.c_char_p, ctypes.c_char_p, VP, CI, VP, CI, VP, CI]),
    "hsfft_fill_complex": (CI, [VP, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64]),
    "hsfft_fill_real": (CI, [VP, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64]),
    "hsfft_time_batched": (CI, [VP, VP, VP, CI, CI, ctypes.POINTER(ctypes.c_float),
                                ctypes.POINTER(ctypes.c_float), CI]),
    "hsfft_time_r2c_batched": (CI, [VP, VP, VP, CI, CI, ctypes.POINTER(ctypes.c_float)]),
    "hsfft_time_exec_host": (CI, [VP, VP, VP, CI, CI, CI, ctypes.POINTER(ctypes.c_double)]),
    "hsfft_exec_multi": (CI, [VP, VP, VP, CI, CI]),
    "hsfft_bench_copy": (CI, [VP, VP, ctypes.c_size_t, CI, ctypes.POINTER(ctypes.c_float)]),
    "hsfft_bluestein_fallbacks": (ctypes.c_longlong, []),
    "hsfft_thread_streams_created": (ctypes.c_longlong, []),
    "hsfft_count_diff_words": (CI, [VP, VP, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64)]),
}

HSFFT_ERR_ARG, HSFFT_ERR_DEVICE, HSFFT_ERR_NOMEM = -1, -2, -3  # include/hsfft_gpu.h

STRUCT_TWIDDLE_OFFSET = 272  # offsetof(struct fft_set, twiddle), include/highspeedFFT.h

_lib = None


class HsfftError(RuntimeError):
    pass


def lib():
    """Load lib/libhsfft.so once and bind every public symbol."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HsfftError(f"{LIB_PATH} not built: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(VP) if isinstance(a, np.ndarray) else VP(a)


def check(rc, what="hsfft"):
    if rc < 0:
        raise HsfftError(f"{what} failed ({rc}): {lib().hsfft_last_error().decode()}")
    return rc


def device_count():
    return lib().hsfft_device_count()


class Plan:
    """fft_object wrapper (fft_init / free_fft)."""

    def __init__(self, n, sgn=1):
        self.n, self.sgn = n, sgn
        self.ptr = lib().fft_init(n, sgn)
        if not self.ptr:
            raise HsfftError(f"fft_init({n}, {sgn}) returned NULL")

    def header(self):
        hdr = (ctypes.c_int * 68).from_address(self.ptr)
        lf = hdr[66]
        return dict(N=hdr[0], sgn=hdr[1], factors=[hdr[2 + i] for i in range(lf)], lf=lf, lt=hdr[67])

    def twiddles(self):
        h = self.header()
        m = int(np.prod(h["factors"])) if h["factors"] else 1
        n = max(m - 1, 0)
        raw = (ctypes.c_double * (2 * n)).from_address(self.ptr + STRUCT_TWIDDLE_OFFSET)
        return np.frombuffer(bytes(raw), dtype=np.complex128).copy()

    def num_passes(self):
        return check(lib().hsfft_plan_num_passes(self.ptr), "num_passes")

    def exec(self, x, out=None):
        """drop-in fft_exec on host numpy arrays (staged through HBM)."""
        x = np.ascontiguousarray(x, dtype=np.complex128)
        y = np.zeros_like(x) if out is None else out
        lib().fft_exec(self.ptr, _ptr(x), _ptr(y))
        return y

    def close(self):
        if self.ptr:
            lib().free_fft(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RealPlan:
    def __init__(self, n, sgn=1):
        self.n, self.sgn = n, sgn
        self.ptr = lib().fft_real_init(n, sgn)
        if not self.ptr:
            raise HsfftError("fft_real_init failed")

    def r2c(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.n, dtype=np.complex128)
        lib().fft_r2c_exec(self.ptr, _ptr(x), _ptr(y))
        return y

    def c2r(self, X):
        X = np.ascontiguousarray(X, dtype=np.complex128)
        y = np.zeros(self.n, dtype=np.float64)
        lib().fft_c2r_exec(self.ptr, _ptr(X), _ptr(y))
        return y

    def close(self):
        if self.ptr:
            lib().free_real_fft(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBuffer:
    """HBM allocation through hsfft_malloc (no torch involved)."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.ptr = lib().hsfft_malloc(self.nbytes)
        if not self.ptr:
            raise HsfftError(f"hsfft_malloc({self.nbytes}) failed: {lib().hsfft_last_error().decode()}")

    @classmethod
    def from_array(cls, a):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        check(lib().hsfft_memcpy_h2d(b.ptr, _ptr(a), a.nbytes), "h2d")
        return b

    def to_array(self, dtype, count=None, offset_bytes=0):
        dt = np.dtype(dtype)
        count = (self.nbytes - offset_bytes) // dt.itemsize if count is None else count
        out = np.empty(count, dtype=dt)
        check(lib().hsfft_memcpy_d2h(_ptr(out), VP(self.ptr + offset_bytes), out.nbytes), "d2h")
        return out

    def fill_zero(self):
        check(lib().hsfft_memset(self.ptr, 0, self.nbytes), "memset")

    def free(self):
        if self.ptr:
            lib().hsfft_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceView:
    """a byte offset into a DeviceBuffer (not owning; never freed)"""

    def __init__(self, buf, offset_bytes):
        self.ptr = buf.ptr + int(offset_bytes)
        self.nbytes = buf.nbytes - int(offset_bytes)


def exec_batched(plan, d_in, d_out, batch):
    return check(lib().hsfft_exec_batched(plan.ptr, VP(d_in.ptr), VP(d_out.ptr), batch), "exec_batched")


def exec_batched_host(plan, x, out=None):
    """c2c of host rows x (batch, N) complex128 through hsfft_exec_batched_host"""
    x = np.ascontiguousarray(x, dtype=np.complex128)
    out = np.empty_like(x) if out is None else out
    batch = x.shape[0] if x.ndim == 2 else 1
    check(lib().hsfft_exec_batched_host(plan.ptr, _ptr(x), _ptr(out), batch), "exec_batched_host")
    return out


def r2c_batched(rplan, d_in, d_out, batch):
    return check(lib().hsfft_r2c_batched(rplan.ptr, VP(d_in.ptr), VP(d_out.ptr), batch), "r2c_batched")


def r2c_batched_compact(rplan, d_in, d_out, batch):
    return check(lib().hsfft_r2c_batched_compact(rplan.ptr, VP(d_in.ptr), VP(d_out.ptr), batch),
                 "r2c_batched_compact")


def c2r_batched(rplan, d_in, d_out, batch):
    return check(lib().hsfft_c2r_batched(rplan.ptr, VP(d_in.ptr), VP(d_out.ptr), batch), "c2r_batched")


def fill_complex(d, count, seed, offset=0):
    return check(lib().hsfft_fill_complex(VP(d.ptr), count, seed, offset), "fill_complex")


def fill_real(d, count, seed, offset=0):
    return check(lib().hsfft_fill_real(VP(d.ptr), count, seed, offset), "fill_real")


def synchronize():
    return check(lib().hsfft_synchronize(), "synchronize")


def finalize():
    """hsfft_finalize(): release every device object the library holds (before process exit)"""
    return check(lib().hsfft_finalize(), "finalize")


def set_twiddle_mode(mode):
    return check(lib().hsfft_set_twiddle_mode({"reference": 0, "exact": 1}.get(mode, mode)), "twiddle_mode")


def time_batched(plan, d_in, d_out, batch, iters, max_pass=16):
    ms = ctypes.c_float(0.0)
    pms = (ctypes.c_float * max_pass)()
    check(lib().hsfft_time_batched(plan.ptr, VP(d_in.ptr), VP(d_out.ptr), batch, iters, ctypes.byref(ms), pms,
                                   max_pass), "time_batched")
    return ms.value, [pms[i] for i in range(max_pass)]


def bench_copy(d_src, d_dst, nbytes, iters):
    ms = ctypes.c_float(0.0)
    check(lib().hsfft_bench_copy(VP(d_src.ptr), VP(d_dst.ptr), nbytes, iters, ctypes.byref(ms)), "bench_copy")
    return ms.value


def count_diff_words(d_a, d_b, nbytes):
    """8-byte words that differ between two device buffers (on the GPU)"""
    c = ctypes.c_uint64(0)
    check(lib().hsfft_count_diff_words(VP(d_a.ptr), VP(d_b.ptr), nbytes, ctypes.byref(c)), "count_diff_words")
    return c.value


def time_r2c_batched(rplan, d_in, d_out, batch, iters):
    ms = ctypes.c_float(0.0)
    check(lib().hsfft_time_r2c_batched(rplan.ptr, VP(d_in.ptr), VP(d_out.ptr), batch, iters, ctypes.byref(ms)),
          "time_r2c_batched")
    return ms.value
