"""In-process A/B of environment knobs on ONE set of device buffers (measurement tool).

Fresh allocations land in fast or slow memory from call to call (allocation
lottery), so comparing two bench runs compares placements as much as kernels.  Here every
variant runs on the same input / output buffers, interleaved round by round; the library reads
its knobs per launch, so setting os.environ between calls switches the variant.

  python tools/ab_env.py --config c3 --var HSFFT_ROW_TWL --values 1,0 --rounds 6
  python tools/ab_env.py --config c5 --values "unset" "HSFFT_R2C_WT=16;HSFFT_R2C_ORDER=0"

A value is either one setting of --var ("unset" removes it) or a ';'-separated list of VAR=VAL
assignments; every variable named anywhere is removed before a variant's own are applied.  The
output buffer is kept as first allocated (bench.probe_placement reports its slice copy rates;
--place selects it by the round-3 probe, bench.place_output, instead).
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "mixed-radix-fast-fourier-transform_amd"))
import hsfft  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (place_output)

CONFIGS = {  # name: (N, rows, real)
    "c2": (1 << 20, 4096, False),
    "c3": (12600, 65536, False),
    "c4": (99991, 8192, False),
    "c5": (1 << 22, 512, True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--var", default="")
    ap.add_argument("--values", required=True, nargs="+",
                    help="comma-separated values of --var ('unset' removes it) or VAR=VAL;VAR=VAL sets")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--place", action="store_true", help="select the output buffer by bench.place_output")
    a = ap.parse_args()
    n, rows, real = CONFIGS[a.config]
    hsfft.lib().hsfft_set_device(0)
    if real:
        p = hsfft.RealPlan(n, 1)
        din = hsfft.DeviceBuffer(rows * n * 8)
        dout = hsfft.DeviceBuffer(rows * n * 16)
        din, dout, rec = bench.place_output(din, dout) if a.place else (din, dout, bench.probe_placement(din, dout))
        hsfft.fill_real(din, rows * n, 0x55)
    else:
        p = hsfft.Plan(n, 1)
        din = hsfft.DeviceBuffer(rows * n * 16)
        dout = hsfft.DeviceBuffer(rows * n * 16)
        din, dout, rec = bench.place_output(din, dout) if a.place else (din, dout, bench.probe_placement(din, dout))
        hsfft.fill_complex(din, rows * n, 0x55)
    print("placement", rec, flush=True)
    vals = [v for arg in a.values for v in (arg.split(",") if "=" not in arg else [arg])]

    def sets(v):
        if "=" in v:
            return dict(kv.split("=", 1) for kv in v.split(";"))
        return {a.var: None if v == "unset" else v}

    names = {k for v in vals for k in sets(v)}

    def run(v, iters):
        for k in names:
            os.environ.pop(k, None)
        for k, x in sets(v).items():
            if x is not None:
                os.environ[k] = x
        if real:
            return hsfft.time_r2c_batched(p, din, dout, rows, iters) / iters
        return hsfft.time_batched(p, din, dout, rows, iters)[0] / iters

    for v in vals:
        run(v, 1)  # warm-up (device state, kernels)
    res = {v: [] for v in vals}
    for r in range(a.rounds):
        for v in (vals if r % 2 == 0 else vals[::-1]):
            ms = run(v, a.iters)
            res[v].append(ms)
        print(f"round {r}: " + "  ".join(f"[{v}] {res[v][-1]:.3f} ms" for v in vals), flush=True)
    for v in vals:
        med = statistics.median(res[v])
        print(f"{a.config} {a.var}={v}: median {med:.3f} ms  ({n * rows / med / 1e6:.2f} GSamples/s)  "
              f"min {min(res[v]):.3f} max {max(res[v]):.3f}", flush=True)


if __name__ == "__main__":
    main()
