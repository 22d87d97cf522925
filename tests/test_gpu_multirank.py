"""The multi-GPU path of bench.py on a real GPU: two ranks launched by
torch.distributed.run (gloo control plane, one process per rank) both select device 0 here
(`LOCAL_RANK % device_count`), each transforms its own contiguous shard of rows through
libhsfft (hsfft_exec_batched) and saves the first and last output row of its shard; every
saved row must equal the oracle's transform of that GLOBAL row bit for bit, which proves the
batch-index sharding (no collective) end to end.  No scaling number is derived from this."""
import os
import subprocess
import sys

import numpy as np
import pytest

import hsfft_testlib as T

import hsfft

pytestmark = pytest.mark.gpu


def test_two_ranks_shard_rows_bit_exact(tmp_path):
    if hsfft.device_count() < 1:
        pytest.skip("no GPU")
    out = tmp_path / "rows"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(T.REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--config", "c2", "--batch", "6",
           "--no-cpu-baseline", "--dump-rows", str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=T.REPO)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert '"n_gpus": 2' in r.stdout
    seen = set()
    for rank in (0, 1):
        z = np.load(out / f"rank{rank}.npz")
        n, seed = int(z["n"]), int(z["seed"])
        for row, g in zip(z["rows"], z["global_rows"]):
            x = T.complex_input(n, seed, batch=1, row0=int(g))
            assert T.bits_equal(row, T.oracle_c2c(x, 1)), (rank, int(g))
            seen.add(int(g))
    assert seen == {0, 5, 6, 11}   # rank 0: rows 0..5, rank 1: rows 6..11
