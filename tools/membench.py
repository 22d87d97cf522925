#!/usr/bin/env python3
"""HBM / Infinity-Cache access-pattern study with copy kernels (development tool).
Variants: U = double2 per thread per iteration (1/4/8), NT = non-temporal load+store."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "mixed-radix-fast-fourier-transform_amd"))
import hsfft  # noqa: E402

L = hsfft.lib()
L.hsd_copy_bench_v.restype = ctypes.c_int
L.hsd_copy_bench_v.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
L.hsfft_set_device(0)
big = hsfft.DeviceBuffer(16 << 30)
big2 = hsfft.DeviceBuffer(16 << 30)
names = ["U1", "U4", "U8", "U1nt", "U4nt", "U8nt"]


def run(mib, variant, grid):
    nbytes = mib << 20
    iters = max(3, min(1000, (32 << 30) // nbytes))
    ms = ctypes.c_float()
    rc = L.hsd_copy_bench_v(big.ptr, big2.ptr, nbytes // 16, iters, variant, grid, ctypes.byref(ms))
    return 2 * nbytes * iters / (ms.value / 1e3) / 1e9 if rc == 0 else -1


for mib in [64, 128, 16384]:
    for v in range(6):
        for grid in [1024, 2048, 4096, 8192, 32768]:
            print(f"{mib:6d} MiB {names[v]:5s} grid {grid:6d}: {run(mib, v, grid):8.1f} GB/s", flush=True)
