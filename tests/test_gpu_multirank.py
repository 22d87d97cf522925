"""The multi-GPU path of bench.py on a real GPU: `bench.py --gpus 2`, started WITHOUT a launcher
(as the driver's own command line may be), starts its two rank processes itself
(torch.distributed.run as a child process; gloo control plane, one process per rank).  Both
ranks select device 0 here (`LOCAL_RANK % device_count`), each transforms its own contiguous
shard of rows through libhsfft and saves the first and last output row of its shard; every
saved row must equal the oracle's transform of that GLOBAL row bit for bit, which proves the
batch-index sharding (no collective) end to end -- for the c2c hot path (config 2) and for the
chunked r2c path (config 5); and four ranks for c2.  No scaling number is derived from this."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import hsfft_testlib as T

import hsfft

pytestmark = pytest.mark.gpu


def run_two_ranks(tmp_path, config, batch, cpu=False, ranks=2):
    if hsfft.device_count() < 1:
        pytest.skip("no GPU")
    out = tmp_path / "rows"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(T.REPO, "bench.py"), "--gpus", str(ranks), "--steps", "2", "--warmup", "1",
           "--config", config, "--batch", str(batch), "--dump-rows", str(out)]
    cmd += ["--cpu-seconds", "1"] if cpu else ["--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=T.REPO)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and lines[0]["n_gpus"] == ranks, r.stdout[-2000:]  # rank 0 only
    assert lines[0]["config"]["global_batch"] == ranks * batch
    return out, lines[0]


def test_two_ranks_shard_rows_bit_exact(tmp_path):
    """... and the N>1 line's own fields: every rank's ms per step and
    roofline figures, the aggregate roofline against 2 x the peak, and the reference timed on the
    host cores by rank 0 in the same run"""
    out, line = run_two_ranks(tmp_path, "c2", 6, cpu=True)
    per = line["per_rank"]
    assert [p["rank"] for p in per] == [0, 1]
    for p in per:
        assert p["ms_per_step"] > 0 and p["event_ms_per_step"] > 0 and 0 < p["frac"] < 1
    agg = line["roofline"]["aggregate"]
    assert agg["peak"] == 16000.0 and 0 < agg["frac"] < 1
    assert line["cpu_baseline"]["value"] > 0 and line["cpu_baseline"]["cores"] >= 1
    seen = set()
    for rank in (0, 1):
        z = np.load(out / f"rank{rank}.npz")
        n, seed = int(z["n"]), int(z["seed"])
        for row, g in zip(z["rows"], z["global_rows"]):
            x = T.complex_input(n, seed, batch=1, row0=int(g))
            assert T.bits_equal(row, T.oracle_c2c(x, 1)), (rank, int(g))
            seen.add(int(g))
    assert seen == {0, 5, 6, 11}   # rank 0: rows 0..5, rank 1: rows 6..11


def test_two_ranks_r2c_chunked_shard_rows_bit_exact(tmp_path):
    """config 5's path (real rows of 2^22, output written chunk by chunk) sharded over two ranks"""
    out, _ = run_two_ranks(tmp_path, "c5", 2)
    seen = set()
    for rank in (0, 1):
        z = np.load(out / f"rank{rank}.npz")
        n, seed = int(z["n"]), int(z["seed"])
        assert str(z["kind"]) == "r2c"
        for row, g in zip(z["rows"], z["global_rows"]):
            x = T.real_input(n, seed, batch=1, row0=int(g))
            assert T.bits_equal(row, T.oracle_r2c(x, 1)), (rank, int(g))
            seen.add(int(g))
    assert seen == {0, 1, 2, 3}


def test_four_ranks_shard_rows_bit_exact(tmp_path):
    """the 4-rank launch (one step towards the driver's 8-GPU run, rehearsed with four ranks on
    the one GPU): contiguous shards of 3 rows each, every rank's first and last row bit-exact,
    four per-rank entries and the aggregate roofline against 4 x the peak"""
    out, line = run_two_ranks(tmp_path, "c2", 3, ranks=4)
    assert [p["rank"] for p in line["per_rank"]] == [0, 1, 2, 3]
    assert line["roofline"]["aggregate"]["peak"] == 32000.0
    seen = set()
    for rank in range(4):
        z = np.load(out / f"rank{rank}.npz")
        n, seed = int(z["n"]), int(z["seed"])
        for row, g in zip(z["rows"], z["global_rows"]):
            x = T.complex_input(n, seed, batch=1, row0=int(g))
            assert T.bits_equal(row, T.oracle_c2c(x, 1)), (rank, int(g))
            seen.add(int(g))
    assert seen == {0, 2, 3, 5, 6, 8, 9, 11}


def test_one_gpu_line_contract(tmp_path):
    """the N = 1 bench line carries the contract's fields: metric / value / unit / n_gpus /
    steps / warmup / ms_per_step / higher_is_better / scaling / vs_baseline / dtype / data /
    config.workload, `roofline` {bound, achieved, peak, unit, frac, traffic} and `cpu_baseline`
    {value, unit, cores, kind, sample} (a small batch: traffic is null off the profiled batch)"""
    if hsfft.device_count() < 1:
        pytest.skip("no GPU")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(T.REPO, "bench.py"), "--steps", "2", "--warmup", "1", "--config", "c2",
           "--batch", "4", "--no-other-configs", "--cpu-seconds", "0.5"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=T.REPO)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0 and d["config"]["workload"]
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0 and "traffic" in rf
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], abs=1e-3)
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["unit"] == "GSamples/s" and cb["cores"] >= 1 and cb["kind"] in ("reference", "port")
    assert cb["sample"]
