"""bench.py --gpus N runs N ranks itself (BASELINE configs[3] multi-GPU line).

Two ranks rehearsed on one GPU over gloo (KRCA_BENCH_BACKEND=gloo, the ranks share the device):
the JSON line reports the ranks of the communicator, and the sharded step (pod-sharded scoring,
one all-gather per PageRank iteration) ranks the same top-10 as one rank.  At N = 2 the line
verifies itself (ranks gathered to rank 0, bit-identical to the oracle; sampled scores of every
rank), whether the PageRank rows are the scoring's uniform ranges or Partition.balanced ones (the
default at N > 1: scores all-gathered once per step), carries the CPU baseline and the per-rank / aggregate roofline, and its correlation leg runs
the pod-sharded krca/corr_dist.py path with its own exactness check.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

ARGS = ["--pods", "20000", "--edges", "400000", "--steps", "2", "--warmup", "1", "--cpu-warmup", "1", "--cpu-runs", "2",
        "--corr-runs", "1"]


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
    two = run_bench(2, ["--profile", "--ppr-partition", "balanced"])
    # the PageRank rows on the scoring's own uniform ranges (no score all-gather)
    two_u = run_bench(2, ["--ppr-partition", "uniform", "--no-corr", "--no-cpu-baseline"])
    # auto: the sharded solve unless the all-gather measured at startup costs more than the margin
    two_a = run_bench(2, ["--no-corr", "--no-cpu-baseline"])
    # every rank solves the whole mesh on the all-gathered scores (no collective inside the solve)
    two_r = run_bench(2, ["--ppr-partition", "replicated", "--no-corr", "--no-cpu-baseline"])
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["world_ranks"] == 2
    assert two["rca_top10"] == one["rca_top10"] == two_u["rca_top10"] == two_r["rca_top10"] == two_a["rca_top10"]
    # the exchange probe and the mode auto took from it
    ex = two_a["ppr_exchange"]
    assert two_a["ppr_exchange_us"] == ex["allgather_us"] > 0 and ex["copy_us"] > 0 and ex["bytes_per_rank"] > 0
    want = "replicated" if ex["iters_x_extra_ms"] > ex["margin_ms"] else "uniform"
    assert two_a["ppr_mode"] == want, ex
    assert two["ppr_mode"] == "balanced" and two_r["ppr_mode"] == "replicated" and one["ppr_exchange_us"] is None
    # the ranking on the spread failure model (untimed C2-size mesh on rank 0), checked against the oracle
    assert one["spread_check"]["top10_identical"] and one["planted_root_recall_spread"] >= 0.8, one["spread_check"]
    assert one["config"]["ranking_key"] == "explained"
    assert two_r["config"]["ppr_bounds"] == [0, 20000]
    # PageRank on Partition.balanced ranges, scores all-gathered (krca.rca.SplitShard; the default at N >= 4)
    assert two["config"]["ppr_bounds"] != two["config"]["shard_bounds"], two["config"]
    assert two_u["config"]["ppr_bounds"] == two_u["config"]["shard_bounds"]
    for vu in (two_u["verify"], two_r["verify"], two_a["verify"]):
        assert vu["ppr_fixed_point_bit_identical"] and vu["top10_identical"] and vu["n_exceed_flags_bit_exact"], vu
    # the profiled solve issues the previous solve's count + 1 steps (networkx's stop rule)
    assert 0 < two["ppr_iters_run"] < 30 and one["ppr_iters_run"] == two["ppr_iters_run"]
    assert two["profile"]["krca_ppr_shard_step_folded"]["launches"] == two["ppr_iters_run"] + 1
    assert two["profile"]["score_exchange"]["launches"] == 1 and two["profile"]["krca_rolling_score"]["launches"] == 1
    for line in (one, two):
        v = line["verify"]
        assert v["ppr_fixed_point_bit_identical"] and v["top10_identical"] and v["n_exceed_flags_bit_exact"], v
        assert v["ranks_gathered"] == line["n_gpus"] and v["score_max_rel_err"] < 1e-5
        assert line["cpu_baseline"]["value"] > 0 and line["roofline"]["traffic"] is not None
        assert line["roofline"]["aggregate"]["peak"] == 8000.0 * line["n_gpus"]
        c = line["corr"]
        assert c["pods"] == 20000 and c["ms"] > 0 and all(c["verify"][key] for key in
                                                          ("counts_exact", "sets_exact", "values_exact", "all_certified"))
    assert two["corr"]["parallelism"].startswith("pod-sharded")
    prof = one["profile"]
    # the profiled step is the folded sequence RcaStep runs: init, n x (folded step, exchange), finish
    n = one["ppr_iters_run"] + 1
    assert prof["krca_ppr_shard_step_folded"]["launches"] == n and prof["krca_rolling_score"]["launches"] == 1
    assert prof["krca_ppr_shard_finish"]["launches"] == 1 and prof["exchange"]["launches"] == n + 1
