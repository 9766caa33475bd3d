#!/usr/bin/env python3
"""Per-phase cycle counters of ppr_step (debug build with -DPPR_TIMING, loaded through KRCA_LIB):
one 30-iteration propagate at C4; prints the per-workgroup cycle split (stage incl. gathers, row
sums, row update, long-row chunks) and the block count spread.  Diagnostic only."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))


def main():
    import torch
    from krca import native, synth
    from krca.rca import RANKING, Comm, DeviceShard, RcaStep
    eng = native.NativeEngine(0)
    P, E = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000, 20 * (int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000)
    m = synth.make_graph(P, n_edges=E, seed=0)
    rng = np.random.default_rng(0)
    s = (np.abs(rng.standard_normal(P)) * 1.5).astype(np.float32)
    s[m.roots] = 12.0
    sh = DeviceShard(eng, None, m.row_ptr, m.col, m.outdeg, P, P, 1, RANKING)
    sh.score_out = {"score": torch.from_numpy(s).cuda()}
    st = RcaStep(sh, Comm(), RANKING, 0)
    st.propagate()
    torch.cuda.synchronize()
    fn = eng.lib.krca_ppr_debug_timing
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(4096 * 5, np.uint64)
    fn(buf.ctypes.data_as(ctypes.c_void_p), 1)
    st.propagate()
    torch.cuda.synchronize()
    fn(buf.ctypes.data_as(ctypes.c_void_p), 1)
    t = buf.reshape(4096, 5).astype(np.float64)
    used = t[:, 4] > 0
    t = t[used]
    tot = t[:, :4].sum(1)
    out = dict(workgroups=int(used.sum()), blocks_per_wg_mean=float(t[:, 4].mean()), blocks_per_wg_max=float(t[:, 4].max()),
               cycles_per_wg_mean=float(tot.mean()) / RANKING.iters, cycles_per_wg_max=float(tot.max()) / RANKING.iters,
               split_mean={k: float(t[:, i].mean()) / RANKING.iters for i, k in enumerate(("stage", "sum", "update", "long"))},
               cycles_per_block={k: float(t[:, i].sum() / t[:, 4].sum()) for i, k in enumerate(("stage", "sum", "update", "long"))})
    if os.environ.get("PPR_TIMING_DUMP"):  # per-workgroup counters + the plan, for a cost-model fit
        np.savez(os.environ["PPR_TIMING_DUMP"], t=buf.reshape(4096, 5), plan=sh.plan.cpu().numpy().reshape(-1, 4))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
