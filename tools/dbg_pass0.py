#!/usr/bin/env python3
"""Dev check: output of the first pass only (HSFFT_DEV_NPASS=1) for G1=1 vs G1=2 runs saved
by separate processes; compares to the exact column DFT.  Usage: dbg_pass0.py N P tag"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mixed-radix-fast-fourier-transform_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import hsfft  # noqa: E402
import hsfft_testlib as T  # noqa: E402

n, P, tag = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
A = n // P
x = T.complex_input(n, 7, batch=1).reshape(1, n)
p = hsfft.Plan(n, 1)
din = hsfft.DeviceBuffer.from_array(x)
dout = hsfft.DeviceBuffer(n * 16)
hsfft.exec_batched(p, din, dout, 1)
hsfft.synchronize()
y = dout.to_array(np.complex128).reshape(A, P)  # [m][u]
cols = x[0].reshape(P, A).T  # column m: x[t*A + m]
for name, ref in (("fwd", np.fft.fft(cols, axis=1)), ("inv", np.fft.ifft(cols, axis=1) * P)):
    err = np.abs(y - ref).max(axis=1) / np.abs(ref).max()
    bad = np.nonzero(err > 1e-9)[0]
    print(tag, name, "max err", err.max(), "bad columns", len(bad), bad[:20])
np.save(os.path.join(REPO, "gpurun_out", f"pass0_{tag}.npy"), y)
