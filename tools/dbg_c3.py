"""debug: config 3 at large batch vs small batch (dev tool)"""
import os, sys
import numpy as np
sys.path.insert(0, "mixed-radix-fast-fourier-transform_amd"); sys.path.insert(0, "tests")
import hsfft, hsfft_testlib as T
n = 12600
hsfft.lib().hsfft_set_device(0)
p = hsfft.Plan(n, 1)
for batch in [16, 1024, 8192, 65536]:
    din = hsfft.DeviceBuffer(batch * n * 16); dout = hsfft.DeviceBuffer(batch * n * 16)
    hsfft.fill_complex(din, batch * n, T.SEEDS[3])
    hsfft.exec_batched(p, din, dout, batch); hsfft.synchronize()
    y = dout.to_array(np.complex128, n, 0)
    x = din.to_array(np.complex128, n, 0)
    xr = T.complex_input(n, T.SEEDS[3], batch=1, row0=0)
    ref = T.oracle_c2c(x, 1)
    print(batch, "input matches generator:", np.array_equal(x, xr), "row0 bit-exact:", T.bits_equal(y, ref),
          "mismatches:", T.mismatches(y, ref), "maxdiff", np.abs(y - ref).max(), flush=True)
    din.free(); dout.free()
