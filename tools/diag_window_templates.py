#!/usr/bin/env python3
"""Diagnostic: the log pass of StreamingRCA.window (side stream, beside the re-rank) against the
same pass run alone -- which containers' line offsets / template histograms differ, if any.
Mirrors tests/test_gpu_stream.py::test_stream_window_log_overlap_and_error_path."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-rca-system_amd")]


def main():
    import torch
    from krca import native, synth
    from krca.agents.logs import pack_documents
    from krca.rca import Config
    from krca.stream import StreamingRCA
    eng = native.NativeEngine()
    P, M, T, W = 2000, 8, 200, 60
    m = synth.make_graph(P, avg_degree=8, seed=31)
    x = synth.make_metrics(P, M, T, window=W, seed=32, roots=m.roots, hop_sets=synth.caller_hops(m, m.roots)).numpy()
    docs = synth.make_log_corpus(P, lines_per_doc=2, seed=33, hazard_rate=0.02)
    docs[5] = "\n".join(["E0101 OOMKilled container worker-7 restarting"] * 5000)
    blob, off = pack_documents(docs)
    text, offd = eng.upload_blob(blob), torch.from_numpy(off).cuda()
    ref = eng.log_scan_device(text, offd)
    ref_t = eng.template_hist_device(ref)
    R = {k: ref[k].cpu().numpy() for k in ("line_start", "line_end", "line_mask", "doc_line0", "doc_lines")}
    RT = {k: ref_t[k].cpu().numpy() for k in ("hash", "n_templates", "tmpl_hash", "tmpl_count")}
    for mode in ("alone-again", "window"):
        if mode == "alone-again":
            s2 = eng.log_scan_device(text, offd)
            t2 = eng.template_hist_device(s2)
        else:
            a = StreamingRCA(eng, m.row_ptr, m.col, m.outdeg, M, Config(window=W), tol=1e-9, max_iter=60)
            o = a.window(torch.from_numpy(x[:W + 40]).cuda(), text, offd)
            s2, t2 = o["logs"], o["logs"]["templates"]
        torch.cuda.synchronize()
        for k, v in R.items():
            g = s2[k].cpu().numpy()
            bad = np.nonzero(g != v)[0]
            print(mode, k, "differ:", len(bad), bad[:10].tolist(), (g[bad[:5]].tolist(), v[bad[:5]].tolist()) if len(bad) else "")
        for k, v in RT.items():
            g = t2[k].cpu().numpy()
            bad = np.nonzero(g != v)[0]
            print(mode, k, "differ:", len(bad), bad[:10].tolist())
            if k == "tmpl_hash" and len(bad):
                d0 = R["doc_line0"]
                docs_bad = np.unique(np.searchsorted(d0, bad, side="right") - 1)
                print("  containers:", docs_bad[:10].tolist(), "n_templates", RT["n_templates"][docs_bad[:10]].tolist())


if __name__ == "__main__":
    main()
