#!/usr/bin/env python3
"""Dev check: one c2c (or r2c) size on the GPU vs the oracle; prints mismatch stats.
Usage: tools/dbg_size.py N [batch] [r2c]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mixed-radix-fast-fourier-transform_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import hsfft  # noqa: E402
import hsfft_testlib as T  # noqa: E402

n = int(sys.argv[1])
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1
real = len(sys.argv) > 3 and sys.argv[3] == "r2c"
if real:
    x = T.real_input(n, 7, batch=batch).reshape(batch, n)
    p = hsfft.RealPlan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(batch * n * 16)
    hsfft.r2c_batched(p, din, dout, batch)
    ref = T.oracle_r2c(x, 1)
else:
    x = T.complex_input(n, 7, batch=batch).reshape(batch, n)
    p = hsfft.Plan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(batch * n * 16)
    hsfft.exec_batched(p, din, dout, batch)
    ref = T.oracle_c2c(x, 1)
hsfft.synchronize()
y = dout.to_array(np.complex128).reshape(batch, -1)
bad = np.nonzero(y.view(np.uint64) != np.asarray(ref).view(np.uint64))
err = np.abs(y - ref).max() / max(1e-300, np.abs(ref).max())
print(f"N={n} batch={batch} real={real} env={[k+'='+v for k, v in os.environ.items() if k.startswith('HSFFT')]} "
      f"passes={getattr(p, 'num_passes', lambda: -1)() if not real else -1} mismatched_words={len(bad[0])} relerr={err:.3e}")
if len(bad[0]):
    idx = np.unique(bad[1] // 2 if False else bad[1])[:16]
    print("  first bad idx:", idx)
