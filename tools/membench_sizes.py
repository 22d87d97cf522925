#!/usr/bin/env python3
"""Copy bandwidth vs buffer size (development tool): is the practical HBM ceiling size-dependent?"""
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
big = hsfft.DeviceBuffer(64 << 30)
big2 = hsfft.DeviceBuffer(64 << 30)
for mib in [512, 1024, 4096, 16384, 65536]:
    for v, name in [(0, "U1"), (1, "U4")]:
        for grid in [4096, 16384, 65536]:
            nbytes = mib << 20
            iters = max(2, min(50, (64 << 30) // nbytes))
            ms = ctypes.c_float()
            rc = L.hsd_copy_bench_v(big.ptr, big2.ptr, nbytes // 16, iters, v, grid, ctypes.byref(ms))
            print(f"{mib:6d} MiB {name} grid {grid:6d}: {2 * nbytes * iters / (ms.value / 1e3) / 1e9:8.1f} GB/s",
                  flush=True)
