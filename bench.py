#!/usr/bin/env python3
"""Headline benchmark: pod·timesteps scored/s + end-to-end RCA top-k latency on a 1M-pod mesh.

BASELINE.json metric, configs[3] shape: synthetic 1M-pod / ~20M-edge mesh, 8 metrics x 1440
steps (46 GB of float32 metrics — it fits one MI355X, so N=1 runs the whole mesh).  One step =
the full RCA hot path (krca/rca.py): rolling z-scores of every pod -> seeded personalized
PageRank (30 fixed-point iterations) -> root-cause top-10 on the host.  Inputs are resident in
HBM before timing; nothing is cached across steps.

Multi-GPU: `python bench.py --gpus N` starts N ranks itself (a `torch.distributed.run` child
process, before anything touches the GPU); under an external launcher (WORLD_SIZE set) it must
equal --gpus.  The mesh is sharded by pod (strong scaling: the same 1M pods over N GPUs), one
all-gather over RCCL per PageRank iteration.  Rank 0 prints ONE JSON line.

Steps are pipelined over two HIP streams (two shard states over the same resident metrics): step
i+1's HBM-bound scoring runs while step i's latency-bound PageRank iterates (the scoring kernels
themselves stay one at a time, ordered by an event), and step i's top-10 is merged on the host
after step i+1 has been enqueued.  Every step still does all of its work;
`e2e_rca_latency_ms` is measured separately, one step at a time.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse(argv=None):
    from krca.rca import RANKING
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--metrics", type=int, default=8)
    ap.add_argument("--tsteps", type=int, default=1440)
    ap.add_argument("--window", type=int, default=RANKING.window)
    ap.add_argument("--iters", type=int, default=RANKING.iters)
    ap.add_argument("--alpha", type=float, default=RANKING.alpha)
    ap.add_argument("--seed-floor", type=float, default=RANKING.seed_floor,
                    help="personalization floor in |z| units (default: krca.rca.Config's scale-aware floor)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-sample-pods", type=int, default=25_000)
    ap.add_argument("--cpu-warmup", type=int, default=3)
    ap.add_argument("--cpu-runs", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run steps back to back on one stream (default: two streams, step i+1's scoring "
                         "overlaps step i's PageRank)")
    ap.add_argument("--profile", action="store_true",
                    help="after the timed steps, one unpipelined step per rank with a HIP event around every "
                         "launch (scoring, PageRank init / step / exchange / reduce, key + top-k) and roctx "
                         "ranges for rocprofv3 --marker-trace; per-kernel times go to the JSON line's 'profile'")
    return ap.parse_args(argv)


def launch_ranks(n, argv):
    """Start n ranks of this script (one per GPU) with torch.distributed.run as a CHILD process —
    nothing in this process has touched the GPU — and return rank 0's launcher exit status."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    log(f"bench: starting {n} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd).returncode


def cpu_model():
    try:
        for ln in subprocess.run(["lscpu"], capture_output=True, text=True, check=True).stdout.splitlines():
            if ln.startswith("Model name:"):
                return ln.split(":", 1)[1].strip()
    except (OSError, subprocess.CalledProcessError):
        pass
    import platform
    return platform.processor()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def profile_step(step, stream, world):
    """One unpipelined RCA step with a HIP event pair around every launch on `stream` (and a roctx
    range per phase): {phase: [ms per launch]} summarised as count / total / mean, plus the step."""
    import torch
    import torch.distributed as dist
    try:
        from torch.cuda import nvtx  # roctx on ROCm builds
        push, pop = nvtx.range_push, nvtx.range_pop
        push("krca.probe")
        pop()
    except Exception:  # noqa: BLE001
        push = pop = lambda *a: None  # noqa: E731
    s, c, cfg = step.s, step.comm, step.cfg
    from krca.rca import step_flags
    rec = []

    def timed(name, fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        push(name)
        a.record()
        fn()
        b.record()
        pop()
        rec.append((name, a, b))

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        timed("krca_rolling_score", s.score)
        timed("krca_ppr_shard_init", lambda: s.init(cfg.alpha, cfg.seed_floor))
        timed("exchange", lambda: c.exchange(s))
        timed("krca_ppr_shard_reduce", lambda: s.reduce(cfg.alpha, cfg.tol, 1))
        for it in range(cfg.iters):
            timed("krca_ppr_shard_step", lambda: s.step(cfg.alpha, step_flags(cfg.tol, it + 1 == cfg.iters)))
            timed("exchange", lambda: c.exchange(s))
            timed("krca_ppr_shard_reduce", lambda: s.reduce(cfg.alpha, cfg.tol, 0))
        timed("key+topk", lambda: s.local_topk(cfg.k))
        t1.record()
    torch.cuda.synchronize()
    out = {}
    for name, a, b in rec:
        out.setdefault(name, []).append(a.elapsed_time(b))
    summ = {k: {"launches": len(v), "total_ms": float(np.sum(v)), "mean_ms": float(np.mean(v))} for k, v in out.items()}
    summ["step_ms"] = t0.elapsed_time(t1)
    summ["note"] = ("HIP events on the launch stream around each call (host launch gaps included in step_ms, "
                    "not in the per-call times); 'exchange' is the all-gather at G > 1, a buffer swap at G = 1")
    return summ


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        log(f"bench: WORLD_SIZE={os.environ.get('WORLD_SIZE')} but --gpus {args.gpus}")
        sys.exit(2)
    import torch
    import torch.distributed as dist

    from krca import native, synth
    from krca.rca import Comm, Config, DeviceShard, RcaStep, shard_graph, shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # KRCA_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices round-robin);
    # the real multi-GPU run is one rank per GPU over RCCL ("nccl")
    backend = os.environ.get("KRCA_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    eng = native.NativeEngine(local)
    cfg = Config(window=args.window, seed_floor=args.seed_floor, alpha=args.alpha, iters=args.iters)
    cfg = cfg.replace(seed_floor=cfg.floor(args.pods, args.metrics))  # resolved once: every rank, the oracle

    # ---- synthetic mesh (host graph, device metrics; not timed) --------------------------
    t0 = time.time()
    mesh = synth.make_graph(args.pods, n_edges=args.edges, seed=args.seed)
    hops = synth.caller_hops(mesh, mesh.roots)
    lo, hi, n_max = shard_range(args.pods, world, rank)
    rp, col, od = shard_graph(mesh.row_ptr, mesh.col, mesh.outdeg, lo, hi)
    x = synth.make_metrics_range(lo, hi, args.metrics, args.tsteps, window=args.window, seed=args.seed,
                                 roots=mesh.roots, hop_sets=hops, device=torch.device("cuda", local))
    n_pipe = 1 if args.no_pipeline else 2
    # one engine per pipeline slot: workspaces are per engine, and the slots run concurrently
    engs = [eng] + [native.NativeEngine(local) for _ in range(n_pipe - 1)]
    shards = [DeviceShard(e, x, rp, col, od, args.pods, n_max, world, cfg) for e in engs]
    steps = [RcaStep(sh, Comm(world, rank), cfg, lo) for sh in shards]
    streams = [torch.cuda.Stream() for _ in range(n_pipe)]
    shard, step = shards[0], steps[0]
    torch.cuda.synchronize()
    log(f"[rank {rank}] mesh N={args.pods} E={mesh.n_edges} shard=[{lo},{hi}) setup {time.time() - t0:.1f}s")

    score_done = [None]  # the scoring kernels run one at a time; only PageRank overlaps them

    def enqueue(i, events=None):
        j = i % n_pipe
        with torch.cuda.stream(streams[j]):
            if score_done[0] is not None:
                streams[j].wait_event(score_done[0])
            if events is not None:
                events[0].record()
            shards[j].score()
            if events is not None:
                events[1].record()
            score_done[0] = torch.cuda.Event()
            score_done[0].record()
            steps[j].propagate()
            return j, *shards[j].local_topk(cfg.k)

    def finish(j, idx, val):
        with torch.cuda.stream(streams[j]):
            return steps[j].merge(idx, val)

    def run_steps(n, events=None, marks=None):
        """marks: host time after each step's top-10 is on the host (per-step spacing)."""
        pending, top = None, None
        for i in range(n):
            cur = enqueue(i, events[i] if events else None)
            if pending is not None:
                top = finish(*pending)
                if marks is not None:
                    marks.append(time.perf_counter())
            pending = cur
        top = finish(*pending)
        if marks is not None:
            marks.append(time.perf_counter())
        return top

    # ---- warmup + timed steps ------------------------------------------------------------
    if args.warmup:
        run_steps(args.warmup)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    marks = [t_start]
    # HIP events on the stream each scoring kernel is launched on
    top_idx, top_key = run_steps(args.steps, ev, marks)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    step_ms = np.diff(np.asarray(marks)) * 1e3  # completion spacing of consecutive steps
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # end-to-end latency of one step (scores -> PageRank -> top-10 on the host), not pipelined
    lat = []
    ev_solo = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for e_solo in ev_solo:
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        with torch.cuda.stream(streams[0]):
            top_idx, top_key = step.run(score_events=e_solo)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t1)
    solo_ms = float(np.median([a.elapsed_time(b) for a, b in ev_solo]))
    latency_ms = float(np.median(lat)) * 1e3
    latency_p95_ms = float(np.percentile(lat, 95)) * 1e3
    if world > 1:
        t = torch.tensor([latency_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        latency_ms = float(t.item())
    score_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    prof = profile_step(step, streams[0], world) if args.profile else None

    # ---- roofline of the dominant kernel (krca_rolling_score) ----------------------------
    n_loc = hi - lo
    bytes_score = 4 * n_loc * args.metrics * args.tsteps + 4 * n_loc * args.metrics + 9 * n_loc
    achieved = bytes_score / (score_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.pmc):
        try:
            pm = json.load(open(args.pmc))
            if pm.get("pods") == args.pods and world == 1:
                traffic = pm.get("krca_rolling_score_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None

    result = None
    if rank == 0:
        value = args.pods * args.tsteps * args.steps / elapsed
        result = {
            "metric": "pod·timesteps scored/s + end-to-end RCA top-k latency (ms), 1M-pod mesh",
            "value": value, "unit": "pod·timesteps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32 (f64 window sums, int64 fixed-point ranks)",
            "data": "synthetic (seeded mesh generator krca/synth.py; no network)",
            "config": {"workload": "C4: synthetic 1M-pod / 20M-edge mesh, 8 metrics x 1440 steps, full RCA step "
                                   "(rolling z-score -> 30-iteration seeded PPR -> top-10), ranking of krca.rca.Config",
                       "pods": args.pods, "edges": mesh.n_edges, "metrics": args.metrics, "tsteps": args.tsteps,
                       "window": args.window, "ppr_iters": args.iters, "alpha": args.alpha,
                       "seed_floor": cfg.seed_floor, "parallelism": f"pod-sharded x{world}"},
            "e2e_rca_latency_ms": latency_ms, "e2e_rca_latency_p95_ms": latency_p95_ms,
            "step_ms_median": float(np.median(step_ms)), "step_ms_p95": float(np.percentile(step_ms, 95)),
            "pipelined_streams": n_pipe,
            "scoring_variant": native.SCORE_VARIANTS[eng.lib.krca_rolling_score_variant(n_loc, args.metrics,
                                                                                      args.tsteps, args.window)],
            "roofline": {"kernel": "krca_rolling_score", "bound": "hbm", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "algorithmic_bytes_per_launch": bytes_score,
                         "avg_launch_ms": score_ms,
                         # the timed steps are pipelined: each scoring launch shares the GPU with the
                         # previous step's PageRank; the same kernel alone (latency steps, same run):
                         "solo_avg_launch_ms": solo_ms,
                         "solo_frac": bytes_score / (solo_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "rca_top10": [int(i) for i in top_idx],
            "world_ranks": world, "backend": backend if world > 1 else None,
            "planted_root_recall": len(set(int(i) for i in top_idx) & set(mesh.roots.tolist())) / len(mesh.roots),
        }

    # ---- verification (not timed): bit-exact PageRank / top-10 vs the C oracle -----------
    if rank == 0 and world == 1 and not args.no_verify:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        score = shard.score_out["score"].cpu().numpy()
        ridx, rf, r = oracle.rca_rank(mesh.row_ptr, mesh.col, mesh.outdeg, score, cfg.alpha, cfg.iters,
                                      cfg.seed_floor, cfg.k)
        dev_r = shard.r[:n_loc].cpu().numpy()
        samp = np.random.default_rng(1).choice(n_loc, size=min(2000, n_loc), replace=False)
        xs = x[:, torch.from_numpy(np.sort(samp)).cuda(), :].cpu().numpy()
        ref = oracle.c_rolling_score(xs, args.window)
        dev = {k: shard.score_out[k][torch.from_numpy(np.sort(samp)).cuda()].cpu().numpy()
               for k in ("n_exceed", "flags", "score")}
        result["verify"] = {
            "ppr_fixed_point_bit_identical": bool(np.array_equal(dev_r, r)),
            "top10_identical": [int(i) for i in ridx] == result["rca_top10"],
            "score_sample_pods": int(len(samp)),
            "n_exceed_flags_bit_exact": bool(np.array_equal(dev["n_exceed"], ref["n_exceed"])
                                             and np.array_equal(dev["flags"], ref["flags"])),
            "score_max_rel_err": float(np.max(np.abs(dev["score"] - ref["score"]) / np.maximum(ref["score"], 1e-6))),
        }

    # ---- CPU baseline: the C restatement on the host cores, bounded sample ---------------
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        ps = min(args.cpu_sample_pods, n_loc)
        xs = x[:, :ps, :].cpu().numpy()
        cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        score = shard.score_out["score"].cpu().numpy()
        t_sc, t_pr = [], []
        for i in range(args.cpu_warmup + args.cpu_runs):  # BASELINE.md §3 protocol
            t1 = time.perf_counter()
            oracle.c_rolling_score(xs, args.window)
            t2 = time.perf_counter()
            oracle.rca_rank(mesh.row_ptr, mesh.col, mesh.outdeg, score, cfg.alpha, cfg.iters, cfg.seed_floor, cfg.k)
            t3 = time.perf_counter()
            if i >= args.cpu_warmup:
                t_sc.append(t2 - t1)
                t_pr.append(t3 - t2)
        # whole step on the CPU at the same mesh size, scoring time scaled from the sample
        t_step = np.asarray(t_sc) * (n_loc / ps) + np.asarray(t_pr)
        med = float(np.median(t_step))
        result["cpu_baseline"] = {
            "value": args.pods * args.tsteps / med, "unit": "pod·timesteps/s", "cores": cores, "kind": "port",
            "sample": f"scoring: oracle/krca_oracle.c on {ps} pods x {args.metrics} x {args.tsteps} "
                      f"(median {np.median(t_sc):.3f} s, scaled x{n_loc / ps:.0f}); PPR+top-10: full {args.pods}-node "
                      f"graph (median {np.median(t_pr):.3f} s); OpenMP threads = {cores}; "
                      f"{args.cpu_warmup} warm-up + {args.cpu_runs} timed runs",
            "ms_per_step": med * 1e3, "ms_per_step_p95": float(np.percentile(t_step, 95)) * 1e3,
            "cpu_model": cpu_model(),
        }
        ref_t = os.path.join(ROOT, "tests", "golden", "ref_cpu_timings.json")
        if os.path.exists(ref_t):  # the reference's own Python, timed in the build container
            rt = json.load(open(ref_t))
            result["cpu_baseline"]["reference_python"] = {
                "where": "build container (reference code never runs on the GPU box): " + rt["host"]["cpu_model"],
                "cores": 1, "timings": {k: {kk: v[kk] for kk in ("median_s", "p95_s", "units", "unit") if kk in v}
                                        for k, v in rt["timings"].items()},
                "note": "the reference has no rolling scoring or PageRank; these are its per-pod threshold "
                        "loop, 13-regex line histogram, SPOF betweenness and C1 comprehensive analysis"}

    if rank == 0 and prof is not None:
        result["profile"] = prof
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
