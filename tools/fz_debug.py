import os, sys, numpy as np
sys.path.insert(0, "mixed-radix-fast-fourier-transform_amd"); sys.path.insert(0, "tests")
import hsfft, hsfft_testlib as T
N = 1 << 20
hsfft.lib().hsfft_set_device(0)
os.environ["HSFFT_FZ_DEBUG"] = os.environ.get("DBG", "1")
os.environ["HSFFT_FZ_SPIN"] = os.environ.get("SPIN", "20000")
SG = int(os.environ.get("SGN", "1"))
for batch, r in [(1, 1), (2, 2), (4, 2)]:
    os.environ["HSFFT_FUSED"] = "1"; os.environ["HSFFT_FZ_R"] = str(r)
    x = T.complex_input(N, 5, batch=batch).reshape(batch, N)
    p = hsfft.Plan(N, SG)
    din = hsfft.DeviceBuffer.from_array(x); dout = hsfft.DeviceBuffer(x.nbytes)
    print("batch", batch, "launch", flush=True)
    rc = hsfft.lib().hsfft_exec_batched(p.ptr, din.ptr, dout.ptr, batch)
    print("rc", rc, flush=True)
    rc = hsfft.lib().hsfft_synchronize()
    print("sync rc", rc, hsfft.lib().hsfft_last_error(), flush=True)
    y = dout.to_array(np.complex128).reshape(batch, N)
    print("bits equal", T.bits_equal(y, T.oracle_c2c(x, SG)), flush=True)
