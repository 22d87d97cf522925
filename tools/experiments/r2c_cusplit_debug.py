"""Development aid (not product): the CU-split r2c pipeline of the development build
(HSFFT_R2C_CUSPLIT) call by call at growing batch, each call synchronised and timed, progress
printed at once -- to see where a stall begins and what the split buys per 512 rows."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "mixed-radix-fast-fourier-transform_amd"))
import hsfft  # noqa: E402

n = 1 << 22
hsfft.lib().hsfft_set_device(0)
rp = hsfft.RealPlan(n, 1)
rows_max = 512
din = hsfft.DeviceBuffer(rows_max * n * 8)
dout = hsfft.DeviceBuffer(rows_max * n * 16)
hsfft.fill_real(din, rows_max * n, 0x55)
hsfft.synchronize()
for env in ({}, {"HSFFT_R2C_CUSPLIT": "4", "HSFFT_R2C_SUB": "64", "HSFFT_R2C_WT": "16"}):
    for k in ("HSFFT_R2C_CUSPLIT", "HSFFT_R2C_SUB", "HSFFT_R2C_WT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    for rows in (8, 65, 128, 512, 512):
        t0 = time.perf_counter()
        hsfft.r2c_batched(rp, din, dout, rows)
        hsfft.synchronize()
        print(f"{env or 'default'} rows {rows}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
print("r2c_cusplit_debug: done", flush=True)
