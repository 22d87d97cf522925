"""world_size-2 (gloo, CPU) coverage of bench.py's multi-GPU path: one process per rank,
batch-index sharding (weak scaling, no data-path collective), barrier + max-over-ranks
timing, rank-0-only JSON.  The GPU step is replaced by the CPU oracle (--dry-run), so this
checks the control path, the shard layout and that every rank saw its own rows."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import hsfft_testlib as T

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_bench(nproc, batch, n, launcher=True):
    """launcher: under torch.distributed.run (how the driver starts N ranks); else plain
    `bench.py --gpus N`, which starts its N rank processes itself"""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    args = [os.path.join(REPO, "bench.py"), "--gpus", str(nproc), "--dry-run", "--steps", "2", "--warmup", "1",
            "--batch", str(batch), "--dry-n", str(n)]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}"] + args if launcher else [sys.executable] + args
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return lines[0]


def expected_checksum(n, row0, batch):
    x = T.complex_input(n, 0x5EED0002, batch=batch, row0=row0).reshape(batch, n)
    return float(np.abs(T.oracle_c2c(x, 1)).sum())


@pytest.mark.parametrize("nproc,launcher", [(1, True), (2, True), (2, False)])
def test_bench_multirank_dry_run(nproc, launcher):
    n, batch = 256, 3
    out = run_bench(nproc, batch, n, launcher)
    assert out["n_gpus"] == nproc and out["scaling"] == "weak" and out["per_rank_batch"] == batch
    assert out["row_starts"] == [r * batch for r in range(nproc)]  # disjoint, contiguous shards
    for r in range(nproc):
        assert out["rank_checksums"][r] == pytest.approx(expected_checksum(n, r * batch, batch), rel=1e-12)
    assert out["value"] > 0 and out["ms_per_step"] > 0
    # the N>1 line carries every rank's own numbers, the aggregate roofline
    # and the reference timed on the host cores in the same run (rank 0, after the timed region)
    per = out["per_rank"]
    assert [p["rank"] for p in per] == list(range(nproc))
    for p in per:
        assert p["ms_per_step"] > 0 and p["event_ms_per_step"] > 0 and p["achieved"] > 0 and p["frac"] > 0
    assert max(p["ms_per_step"] for p in per) == pytest.approx(out["ms_per_step"], rel=1e-3)
    agg = out["roofline"]["aggregate"]
    assert agg["peak"] == 8000.0 * nproc and agg["achieved"] > 0
    assert agg["frac"] == pytest.approx(agg["achieved"] / agg["peak"], abs=1e-4)
    cb = out["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("reference", "port") and cb["unit"] == "GSamples/s"


def test_row_range_partition():
    sys.path.insert(0, REPO)
    import bench
    got = [bench.row_range(r, 4096) for r in range(8)]
    assert got[0] == (0, 4096) and all(got[i][1] == got[i + 1][0] for i in range(7)) and got[7][1] == 8 * 4096


def test_world_size_must_match_gpus():
    """under a launcher, --gpus N with WORLD_SIZE != N is refused (a one-GPU timing must not be
    reported as N GPUs, nor the other way round)"""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--dry-run"], cwd=REPO,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in r.stderr
