"""C5 at full size under parity (BASELINE configs[4]; replaces the per-window work of
ref:agents/logs_agent.py:147-151 and ref:agents/metrics_agent.py:88-94): one 1M-pod / 2.5M-line
streaming window on one GPU.

History: 1440 steps of 1M pods x 8 metrics streamed in, a cold PageRank solve (networkx stop rule,
tol 1e-9); then ONE window: 1 new step per pod, 2.5M log lines over 1M containers, warm re-ranking.
Checked:
- stream scores of 20,000 sampled pods == oracle.c_rolling_score over the series so far (flags and
  n_exceed bit-exact, z / score within 1e-5: the same float64 arithmetic);
- 13-bin histograms, line counts and first-3 examples, and template histograms of 20,000 sampled
  containers == the oracle (Python re / str.splitlines, FNV-1a of the template);
- the cold and the warm-started fixed-point ranks bit-identical to the C oracle chain
  (oracle.c_ppr_ex cold, then warm), with the same iteration counts and top-10 (krca.rca.Config's key).
"""
import numpy as np
import pytest
import torch

import oracle
from krca import native, synth
from krca.agents.logs import pack_documents
from krca.rca import Config
from krca.stream import StreamingRCA

pytestmark = pytest.mark.gpu


def test_c5_full_window_1m_pods():
    P, E, M, T, W = 1_000_000, 20_000_000, 8, 1440, 60
    eng = native.NativeEngine()
    mesh = synth.make_graph(P, n_edges=E, seed=0)
    hops = synth.caller_hops(mesh, mesh.roots)
    x = synth.make_metrics_range(0, P, M, T + 1, seed=0, roots=mesh.roots, hop_sets=hops, device="cuda")
    cfg = Config(window=W)
    s = StreamingRCA(eng, mesh.row_ptr, mesh.col, mesh.outdeg, M, cfg, horizon=T, tol=1e-9, max_iter=100)
    s.push_metrics(x[:T])
    top0, _ = s.rerank()
    sc0 = s.shard.score_out["score"].cpu().numpy()
    r0 = s.shard.r[:P].cpu().numpy()
    it0 = s.last_iters
    docs = synth.make_log_corpus(P, lines_per_doc=2.5, seed=1, hazard_rate=0.001)
    blob, off = pack_documents(docs)
    eng.check_log_unicode(blob)
    text = eng.upload_blob(blob)
    offd = torch.from_numpy(off).cuda()
    # ---- the window --------------------------------------------------------------------------
    sc = s.push_metrics(x[T:T + 1])
    scan = s.push_logs(text, offd)
    top, _ = s.rerank()
    torch.cuda.synchronize()
    assert scan["n_lines_total"] > 2_400_000
    rng = np.random.default_rng(3)
    # scores of sampled pods vs the batch oracle over the whole series so far
    samp = np.sort(rng.choice(P, 20_000, replace=False))
    ref = oracle.c_rolling_score(x[:, torch.from_numpy(samp).cuda(), :].cpu().numpy(), W)
    got = {k: v[torch.from_numpy(samp).cuda()].cpu().numpy() for k, v in sc.items()}
    assert np.array_equal(got["flags"], ref["flags"]) and np.array_equal(got["n_exceed"], ref["n_exceed"])
    assert np.allclose(got["score"], ref["score"], rtol=1e-5, atol=1e-6)
    assert np.allclose(got["z_last"], ref["z_last"], rtol=1e-5, atol=1e-6)
    del x
    # logs and templates of sampled containers
    cs = np.sort(rng.choice(P, 20_000, replace=False))
    hist = scan["hist"].cpu().numpy()
    nl = scan["doc_lines"].cpu().numpy()
    ls, le = scan["line_start"].cpu().numpy(), scan["line_end"].cpu().numpy()
    tm = scan["templates"]
    d0 = scan["doc_line0"].cpu().numpy()
    ex = native.example_ids(scan["line_mask"].cpu().numpy(), d0, nl)  # the example bits of the masks
    nt = tm["n_templates"].cpu().numpy()
    th = tm["tmpl_hash"].cpu().numpy().view(np.uint64)
    tc = tm["tmpl_count"].cpu().numpy()
    for d in cs:
        n, h, exs = oracle.log_hist(docs[d])
        assert nl[d] == n and hist[d].tolist() == h, d
        for c in range(13):
            got_ex = [blob[ls[i]:le[i]].decode("utf-8", "surrogatepass") for i in ex[d, c] if i >= 0]
            assert got_ex == exs[c], (d, c)
        want = oracle.template_hist(docs[d])
        assert list(zip(th[d0[d]:d0[d] + nt[d]].tolist(), tc[d0[d]:d0[d] + nt[d]].tolist())) == want, d
    # ranks: cold then warm, bit-identical to the C oracle chain
    fl = cfg.floor(P, M)
    o = oracle.c_ppr_ex(mesh.row_ptr, mesh.col, mesh.outdeg, sc0, cfg.alpha, 100, 1e-9, fl)
    r_ref, it_ref = o["r"], o["it"]
    assert np.array_equal(r0, r_ref) and it0 == it_ref
    ridx, _ = oracle.topk_ref(oracle.rca_keys_from(o, sc0, fl, mesh.row_ptr, mesh.col), cfg.k)
    assert [int(i) for i in top0] == [int(i) for i in ridx]
    score = sc["score"].cpu().numpy()
    o = oracle.c_ppr_ex(mesh.row_ptr, mesh.col, mesh.outdeg, score, cfg.alpha, 100, 1e-9, fl, r_start=r_ref)
    r_ref, it = o["r"], o["it"]
    assert np.array_equal(s.shard.r[:P].cpu().numpy(), r_ref) and s.last_iters == it
    ridx, _ = oracle.topk_ref(oracle.rca_keys_from(o, score, fl, mesh.row_ptr, mesh.col), cfg.k)
    assert [int(i) for i in top] == [int(i) for i in ridx]
    print(f"C5 window: {scan['n_lines_total']} lines, cold solve {it0} iterations, warm {it}")
