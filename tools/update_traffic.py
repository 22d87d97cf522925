#!/usr/bin/env python3
"""Write profiles/pmc_traffic.json's entry for one bench config from a tools/prof_summary.py
JSON: the dominant kernel (`--kernel` substring) and the other kernels with HBM bytes.
Usage: tools/update_traffic.py [--launches-per-step K] <summary.json> <config> <kernel-substring> <batch>
       <algorithmic bytes> <source file> <profile tag> [step-kernel-substring ...]
The step total (`hbm_bytes_per_step`) sums the per-launch bytes of the dominant kernel and of
every kernel matching one of the step-kernel substrings (the launches of one call), times K
when one bench step is K such calls (c5: 4096 rows in 512-row calls)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    lps = 1
    if sys.argv[1] == "--launches-per-step":
        lps = int(sys.argv[2])
        del sys.argv[1:3]
    summ, cfg, ksub, batch, alg, source, tag = sys.argv[1:8]
    s = json.load(open(summ))
    dom = [k for k in s if ksub in k and "hbm_bytes_corrected" in s[k]]
    if len(dom) != 1:
        sys.exit(f"kernel substring {ksub!r} matches {dom}")
    k = dom[0]
    e = s[k]
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    cur = json.load(open(path)) if os.path.exists(path) else {}
    cur[cfg] = {
        "kernel": k,
        "batch": int(batch),
        "hbm_bytes_per_launch": int(e["hbm_bytes_corrected"]),
        "fetch_size_kib": e["FETCH_SIZE"],
        "write_size_kib": e["WRITE_SIZE"],
        "avg_ms": e["avg_ms"],
        "algorithmic_bytes_per_launch": int(alg),
        "other_kernels": {o: {"hbm_bytes_per_launch": int(v["hbm_bytes_corrected"]), "avg_ms": v.get("avg_ms")}
                          for o, v in s.items() if o != k and "hbm_bytes_corrected" in v and v.get("calls", 0) > 1},
        "launches_per_step": lps,
        "hbm_bytes_per_step": lps * (int(e["hbm_bytes_corrected"]) + sum(
            int(v["hbm_bytes_corrected"]) for o, v in s.items()
            if o != k and "hbm_bytes_corrected" in v and any(sub in o for sub in sys.argv[8:]))),
        "step_kernels": [k] + [o for o in s if o != k and "hbm_bytes_corrected" in s[o] and any(sub in o for sub in sys.argv[8:])],
        "method": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of `python3 bench.py "
                  f"--no-cpu-baseline` (tools/profile.sh {tag}); bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 "
                  "(gfx950 FETCH_SIZE reports half of a wide streaming read, MI355X_MICROARCH.md HBM section); "
                  "FETCH/WRITE count L2<->fabric traffic with Infinity Cache hits included",
        "source": source,
    }
    json.dump(cur, open(path, "w"), indent=1)
    print(json.dumps(cur[cfg], indent=1))


if __name__ == "__main__":
    main()
