#!/usr/bin/env python3
"""Why did a captured PageRank solve replay wrong with the HIP runtime's graph packet capture on
?  Runs tests/test_gpu_kernels.py::test_rca_graph_replay_after_eager_launches'
scenario with the diagnosis build (lib/dbg/libkrca_gdbg.so, `make -C kubernetes-rca-system_amd/csrc gdbg`:
ppr_init / ppr_step / ppr_finish printf their arguments and the ctl header from workgroup 0) and
packet capture left at the runtime's default, so each replay's kernel arguments can be compared
with the eager solve's and the first replay's.  Finding (R6a): at the bad replay every
kernel argument was the first replay's, but the ctl header held another kernel's argument words --
the captured hipMemsetAsync that zeroes it had replayed stale bytes; with the solve's zeroing done by
kernels (round 6) every replay is exact (R6b: 300 and 5000 torch or libkrca launches between).

  KRCA_LIB=kubernetes-rca-system_amd/lib/dbg/libkrca_gdbg.so python tools/graph_replay_probe.py [--launches 300]

If the second replay's printed pointers / iteration numbers differ from the first's, the packets'
kernel arguments were overwritten (a kernarg pool reused by later eager launches); if they match
but the ctl header or ranks differ, a device buffer was.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=300)
    ap.add_argument("--junk", choices=("torch", "krca"), default="torch")
    ap.add_argument("--pods", type=int, default=20000)
    a = ap.parse_args()
    import torch

    import krca.rca as rca
    from krca import native, synth
    print("DEBUG_CLR_GRAPH_PACKET_CAPTURE =", os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE"), flush=True)
    print("library:", native.library_info(), flush=True)
    eng = native.NativeEngine(0)
    n = a.pods
    m = synth.make_graph(n, avg_degree=20, seed=5)
    cfg = rca.Config(iters=30, tol=0.0)
    rp, col, od = rca.shard_graph(m.row_ptr, m.col, m.outdeg, 0, n)
    x0 = synth.make_metrics(n, 8, 300, window=60, seed=1, roots=m.roots, hop_sets=synth.caller_hops(m, m.roots)).cuda()

    def mark(s):
        torch.cuda.synchronize()
        sys.stdout.flush()
        print(f"==== {s}", flush=True)

    xe = x0.clone()
    st_e = rca.RcaStep(rca.DeviceShard(eng, xe, rp, col, od, n, n, 1, cfg), rca.Comm(), cfg, 0)
    mark("eager solve")
    st_e.run()
    ref = st_e.s.r[:n].clone()
    mark("eager done")
    xg = x0.clone()
    st_g = rca.RcaStep(rca.DeviceShard(eng, xg, rp, col, od, n, n, 1, cfg), rca.Comm(), cfg, 0, graph=True)
    mark("first run (eager warm-up, capture, replay 1)")
    st_g.run()
    mark("replay 1 done")
    ok1 = torch.equal(st_g.s.r[:n], ref)
    print("replay 1 equals eager:", ok1, flush=True)
    junk = torch.zeros(64, device="cuda")
    if a.junk == "torch":
        for _ in range(a.launches):
            junk.add_(1.0)
    else:  # libkrca launches of another kind (top-k over a small vector)
        v = torch.rand(4096, device="cuda")
        for _ in range(a.launches):
            eng.topk_device(v, 10)
    mark(f"after {a.launches} {a.junk} launches: replay 2")
    st_g.run()
    mark("replay 2 done")
    ok2 = torch.equal(st_g.s.r[:n], ref)
    diff = int((st_g.s.r[:n] != ref).sum())
    print("replay 2 equals eager:", ok2, "differing ranks:", diff, flush=True)
    print("RESULT", dict(replay1=ok1, replay2=ok2, launches=a.launches, junk=a.junk,
                         packet_capture=os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE")), flush=True)


if __name__ == "__main__":
    main()
