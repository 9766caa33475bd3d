"""bench.py --gpus N runs N ranks itself (BASELINE configs[3] multi-GPU line).

Two ranks rehearsed on one GPU over gloo (KRCA_BENCH_BACKEND=gloo, the ranks share the device):
the JSON line reports the ranks of the communicator, and the sharded step (pod-sharded scoring,
one all-gather per PageRank iteration) ranks the same top-10 as one rank.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

ARGS = ["--pods", "20000", "--edges", "400000", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]


def run_bench(n, extra=()):
    env = dict(os.environ, KRCA_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *ARGS, *extra], env=env,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_gpus_2_runs_two_ranks():
    one = run_bench(1, ["--profile"])
    two = run_bench(2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["world_ranks"] == 2
    assert two["rca_top10"] == one["rca_top10"]
    assert one["verify"]["ppr_fixed_point_bit_identical"] and one["verify"]["top10_identical"]
    prof = one["profile"]
    assert prof["krca_ppr_shard_step"]["launches"] == 30 and prof["krca_rolling_score"]["launches"] == 1
