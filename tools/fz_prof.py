"""Fused 2^20 launch: per-queue time breakdown from the HSFFT_FZ_DEBUG trace (dev tool)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "mixed-radix-fast-fourier-transform_amd"))
import hsfft  # noqa: E402

N = 1 << 20
batch = int(os.environ.get("BATCH", "512"))
hsfft.lib().hsfft_set_device(0)
p = hsfft.Plan(N, 1)
din = hsfft.DeviceBuffer(batch * N * 16)
dout = hsfft.DeviceBuffer(batch * N * 16)
hsfft.fill_complex(din, batch * N, 7)
os.environ["HSFFT_FUSED"] = "1"
for it in range(3):
    os.environ["HSFFT_FZ_DEBUG"] = "1" if it == 2 else "0"
    hsfft.exec_batched(p, din, dout, batch)
    hsfft.synchronize()
print("done", flush=True)
