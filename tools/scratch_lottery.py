"""c5 step time over fresh placements of the library's scratch pool (measurement tool): fixed,
placement-checked input / output buffers; every round frees the pool (hsfft_release_scratch),
so the next call allocates its 16 GiB intermediate anew."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "mixed-radix-fast-fourier-transform_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hsfft  # noqa: E402
import bench  # noqa: E402


def main():
    n, rows = 1 << 22, 512
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    hsfft.lib().hsfft_set_device(0)
    p = hsfft.RealPlan(n, 1)
    din, dout = hsfft.DeviceBuffer(rows * n * 8), hsfft.DeviceBuffer(rows * n * 16)
    din, dout, rec = bench.place_output(din, dout)
    print("placement", rec, flush=True)
    hsfft.fill_real(din, rows * n, 0x55)
    ts = []
    for r in range(rounds):
        hsfft.check(hsfft.lib().hsfft_release_scratch(), "release_scratch")
        ms = hsfft.time_r2c_batched(p, din, dout, rows, 3) / 3
        ts.append(ms)
        print(f"scratch allocation {r}: {ms:.3f} ms ({n * rows / ms / 1e6:.2f} GSamples/s)", flush=True)
    print(f"median {statistics.median(ts):.3f} min {min(ts):.3f} max {max(ts):.3f}", flush=True)


if __name__ == "__main__":
    main()
