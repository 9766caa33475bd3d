#!/usr/bin/env python3
"""Per-phase cycle split of log_index_match (KRCA_LOG_FUSED=1/2) or log_index_lines (the default)
from a -DLOG_TIMING build loaded through KRCA_LIB: one
1M-container scan of the C5 corpus, then the per-workgroup sums of thread 0's clock between the
kernel's barriers -- ticket, A (loads, container starts, line-start bits, chunk counts), scan +
aggregate, look-back, list build, DFA walk, writes -- per tile.  Diagnostic only."""
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
    from krca.agents.logs import pack_documents
    eng = native.NativeEngine(0)
    docs = synth.make_log_corpus(int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000, lines_per_doc=2.5, seed=1,
                                 hazard_rate=0.001)
    blob, off = pack_documents(docs)
    tb, toff = eng.upload_blob(blob), torch.from_numpy(off).cuda()
    fn = eng.lib.krca_log_debug_timing
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(1024 * 16, np.uint64)
    eng.log_scan_device(tb, toff, validate=False)
    eng.log_scan_device(tb, toff, validate=False)
    torch.cuda.synchronize()
    fn(buf.ctypes.data_as(ctypes.c_void_p), 1)
    eng.log_scan_device(tb, toff, validate=False)
    torch.cuda.synchronize()
    fn(buf.ctypes.data_as(ctypes.c_void_p), 1)
    t = buf.reshape(1024, 16).astype(np.float64)
    t = t[t[:, 7] > 0]
    fused = int(os.environ.get("KRCA_LOG_FUSED", "0")) != 0
    names = (["ticket", "A_tail_barrier", "scan_agg", "lookback", "list", "walk", "write", "-", "A_issue_loads",
              "A_container_starts", "A_pieces"] if fused else
             ["ticket_container_starts", "loads_flags", "scan", "lookback", "writes", "-", "-"])
    tiles = t[:, 7].sum()
    per_tile = {n: float(t[:, i].sum() / tiles) for i, n in enumerate(names) if n != "-"}
    out = dict(kernel="log_index_match" if fused else "log_index_lines", bytes=len(blob), workgroups=int(len(t)), tiles=int(tiles), cycles_per_tile=per_tile,
               total_cycles_per_wg_mean=float((t[:, :7].sum(1) + t[:, 8:].sum(1)).mean()),
               total_cycles_per_wg_max=float((t[:, :7].sum(1) + t[:, 8:].sum(1)).max()))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
