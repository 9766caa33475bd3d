/*
 * krca.h — C-ABI of libkrca.so, the MI355X (gfx950) numeric core behind the RCA agents.
 *
 * The reference (vobbilis/kubernetes-rca-system) is pure Python, so there is no FFI of its own
 * to mirror; these entry points replace the per-pod Python loops of its non-LLM agents and are
 * bound from Python with ctypes (kubernetes-rca-system_amd/krca/native.py; INTEGRATION.md shows
 * the binding a maintainer would add to the reference).  Each entry cites the reference code
 * whose loop it replaces.
 *
 * Conventions:
 *  - every buffer argument is a caller-owned DEVICE pointer unless the name ends in _host;
 *  - `stream` is a hipStream_t (NULL = default stream); calls are asynchronous unless noted;
 *  - no allocation on the hot path: scratch comes from caller workspaces sized by the
 *    *_workspace_size / *_num_* helpers;
 *  - return 0 on success, a negative errno-style code on failure; krca_last_error() returns a
 *    thread-local message; no C++ exception crosses the ABI;
 *  - re-entrant per stream; integer outputs are deterministic (no order-dependent reductions).
 */
#ifndef KRCA_H
#define KRCA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KRCA_OK 0
#define KRCA_EINVAL (-22)
#define KRCA_ENOMEM (-12)
#define KRCA_EDEVICE (-5) /* HIP runtime error */
#define KRCA_ENOTCONV (-70) /* PageRank did not converge within max_iter */

#define KRCA_NCAT 13 /* log error categories, ref:agents/logs_agent.py:20-34 */

/* flag bits of krca_usage_flags / krca_rolling_score (ref:agents/metrics_agent.py:93,101,140,148) */
#define KRCA_F_CPU80 1u
#define KRCA_F_CPU90 2u
#define KRCA_F_MEM80 4u
#define KRCA_F_MEM90 8u

int krca_version(void);
const char* krca_last_error(void);
int krca_device_count(int* n_host);

/* Kernel-development A/B switches: KRCA_SCORE_IMPL, KRCA_SCORE_CHUNK, KRCA_SCORE_NT, KRCA_PPR_GRID, KRCA_PPR_DICT,
 * KRCA_LOG_IMPL, KRCA_GROUP_IMPL, KRCA_CORR_DEBUG, KRCA_CORR_RS_GRID, KRCA_CORR_BATCH, KRCA_CORR_AMB_TILE,
 * KRCA_PPR_FUSE, KRCA_PPR_NT, KRCA_PPR_XCD, KRCA_LOG_FUSED, KRCA_CORR_RS_GROUP, KRCA_CORR_SIDE, KRCA_CORR_RS_Q16,
 * KRCA_CORR_CAPC, KRCA_CORR_KM_EXTRA, KRCA_CORR_RSG_GRID, KRCA_CORR_PROJ, KRCA_CORR_PERSIST.  Initialised once from the environment variables
 * of the same names when the library loads; launchers never call getenv.  Process-global, not
 * thread-safe (set them before launching work).  Unknown names: KRCA_EINVAL. */
int krca_tune_set(const char* name, int32_t value);
int krca_tune_get(const char* name, int32_t* value_host);

/* ---- a1/a2: instantaneous usage thresholds ------------------------------------------------
 * Replaces the pod loops of MetricsAgent._analyze_cpu_usage / _analyze_memory_usage
 * (ref:agents/metrics_agent.py:88-94, 135-141): flags[p] gets KRCA_F_CPU80 iff usage[p][0] > 80,
 * KRCA_F_CPU90 iff > 90, KRCA_F_MEM80 / KRCA_F_MEM90 likewise for usage[p][1] (strict, float32). */
int krca_usage_flags(const float* usage /*[P][2]*/, int64_t P, uint8_t* flags /*[P]*/, void* stream);

/* ---- a5: rolling z-score anomaly scoring (new primitive; plugs in at
 * ref:agents/metrics_agent.py:44-47).  x is time-major [T][P][M] float32 (series s = p*M+m).
 * For t in [W, T), over the trailing window x[t-W..t-1] (float64 sliding sums s1, s2 in a fixed
 * order): A = W*x_t - s1, B = W*s2 - s1^2 (= W^2 var, ddof 0), z = A/sqrt(B) = (x_t - mean)/std;
 * exceed(t) = B > 1e-12*W^2 && A^2 > z_thr^2 * B.   Outputs:
 *   z_last[p][m] = z at t = T-1 (0 if B <= 1e-12*W^2),   score[p] = max_m |z_last|,
 *   n_exceed[p]  = sum over m, t of exceed(t) (bit-exact vs oracle/krca_oracle.c),
 *   flags[p]     = KRCA_F_* of x[T-1][p][0] (CPU %) and x[T-1][p][1] (memory %) if M >= 2.
 * M must be a power of two <= 64.  Samples are expected finite (a missing sample is the caller's
 * to impute); a NaN / Inf never faults and gives what oracle/krca_oracle.c gives (tested). */
int krca_rolling_score(const float* x, int64_t P, int32_t M, int32_t T, int32_t W, float z_thr,
                       float* z_last, float* score, int32_t* n_exceed, uint8_t* flags, void* stream);
/* which kernel krca_rolling_score launches for these sizes (host query, no device work):
 * KRCA_SCORE_PIPE software-pipelined chunks (the default), KRCA_SCORE_PIPE_ROWS the same with one
 * buffer descriptor per row (series counts past the 2^31-byte descriptor range),
 * KRCA_SCORE_RING plain loads, KRCA_SCORE_RING_BUF W-block buffer loads, KRCA_SCORE_REREAD any W. */
#define KRCA_SCORE_PIPE 0
#define KRCA_SCORE_RING 1
#define KRCA_SCORE_RING_BUF 2
#define KRCA_SCORE_REREAD 3
#define KRCA_SCORE_PIPE_ROWS 4
#define KRCA_SCORE_LDS 5 /* A/B (KRCA_SCORE_IMPL=5, W = 60): rows staged by LDS-DMA, 1 KiB per wave instruction */
int krca_rolling_score_variant(int64_t P, int32_t M, int32_t T, int32_t W);

/* ---- a11/a12: 13-category log histograms (ref:agents/logs_agent.py:124-181) ----------------
 * text = UTF-8 bytes of D container logs, container d = text[doc_off[d], doc_off[d+1]).
 * Contract: doc_off[0] == 0, doc_off[D] == nbytes, doc_off non-decreasing, each container valid
 * UTF-8 on its own (the host wrappers check the offsets; off-contract offsets are clamped on the
 * device so they cannot fault, but the results are then unspecified).
 * Lines are str.splitlines() lines; a line is in category c iff
 * re.search(pattern_c, line, re.IGNORECASE) (compiled DFA, csrc/log_dfa_tables.h).
 * Two phases (the line count is data-dependent):
 *   krca_log_index: per-chunk line-start counts + scan into block_base (workspace of
 *                   krca_log_index_size(nbytes) int64) and *n_lines (device int64).
 *   krca_log_match: (same workspace; it also keeps the first line id of every 256-byte chunk
 *                   there) per line start/end byte offsets and 13-bit mask; per container the line
 *                   count and the 13-bin histogram — atomics-free segmented reduction.  The first
 *                   three matching lines per bin (the reference's evidence, :159-163) are marked in
 *                   the line masks: bit 16 + c of line_mask[l] is set iff line l is one of the first
 *                   three lines of its container in category c (bits 0-12: the categories).
 *                   examples (nullable) additionally receives them as a dense id table
 *                   [D][13][3] (-1 when fewer). */
/* The compiled matcher's identity: the Unicode version of the interpreter that generated the
 * tables (re.IGNORECASE folds, \d, str.splitlines separators; non-ASCII text matches the
 * reference exactly only under that version) and gen_log_dfa.pattern_digest of the 13 patterns
 * (krca/agents/logs.py refuses an edited LogsAgent.error_patterns that no longer matches it). */
const char* krca_log_dfa_unicode(void);
uint64_t krca_log_dfa_digest(void);
int64_t krca_log_index_size(int64_t nbytes);
int krca_log_index(const uint8_t* text, int64_t nbytes, const int64_t* doc_off, int64_t ndocs,
                   int64_t* workspace, int64_t* n_lines, void* stream);
int krca_log_match(const uint8_t* text, int64_t nbytes, const int64_t* doc_off, int64_t ndocs,
                   int64_t* workspace, int64_t n_lines,
                   int64_t* line_start /*[L]*/, int64_t* line_end /*[L]*/, uint32_t* line_mask /*[L]*/,
                   int32_t* doc_lines /*[D]*/, int32_t* hist /*[D][13]*/, int32_t* examples /*[D][13][3], nullable*/,
                   int64_t* doc_line0 /*[D], nullable: first line id of each container*/, void* stream);
/* krca_log_scan: krca_log_index + krca_log_match in one call when the caller's line arrays hold
 * line_cap lines (the same loop, ref:agents/logs_agent.py:140-151): the line index is built in ONE
 * pass over the text (decoupled look-back for the line ids), the later kernels read the line count
 * on the device, and the stream is synchronised once, at the end, for *n_lines_host.  When
 * *n_lines_host > line_cap the outputs past the index are not valid: size the arrays and call
 * krca_log_match with the same workspace (the index is kept there). */
int krca_log_scan(const uint8_t* text, int64_t nbytes, const int64_t* doc_off, int64_t ndocs,
                  int64_t* workspace, int64_t line_cap,
                  int64_t* line_start /*[line_cap]*/, int64_t* line_end /*[line_cap]*/, uint32_t* line_mask /*[line_cap]*/,
                  int32_t* doc_lines /*[D]*/, int32_t* hist /*[D][13]*/, int32_t* examples /*[D][13][3], nullable*/,
                  int64_t* doc_line0 /*[D], nullable*/, int64_t* n_lines_host, void* stream);

/* ---- a13: error-template hashing + per-container template histograms (new primitive) ------
 * template(line) = line bytes with every maximal [A-Za-z0-9_] run that contains an ASCII digit or
 * is >= 8 hex digits long replaced by the one byte 0xFF (shown as "<*>"; never in UTF-8 text);
 * hash = FNV-1a-64(template) (csrc/template.hip).
 * krca_template_hash: hash[l] for every line [line_start[l], line_end[l]) (krca_log_match's lines;
 *   fastest when the starts ascend, as there: a workgroup reads its lines through one window from
 *   its first line's start; lines outside that window are read directly, same hash).
 * krca_template_hist: per container d, the distinct hashes of its lines in ascending order and
 *   their counts, written to out_hash/out_count at the container's own line range
 *   [doc_line0[d], doc_line0[d] + n_templates[d]), then 0 in the slots up to doc_line0[d] + doc_lines[d]
 *   (every slot of the line range is written; those of containers above krca_template_max_lines()
 *   by krca_template_hist_huge).  Sort-based.  Containers of <= 8 lines are sorted
 *   in one lane's registers, <= 64 by a wave, <= krca_template_max_lines() by a workgroup, all on
 *   device lists (no host round trip).  workspace: krca_template_hist_ws_size(ndocs) bytes, int32
 *   {mid, big, huge counts, 0 | mid list [D] | big list [D] | huge list [D]}: containers above
 *   krca_template_max_lines() lines are only LISTED (count at int32 [2], ids from int32 [4 + 2D]);
 *   the caller runs krca_template_hist_huge on each. */
int krca_template_hash(const uint8_t* text, int64_t nbytes, const int64_t* line_start, const int64_t* line_end,
                       int64_t n_lines, uint64_t* hash, void* stream);
int64_t krca_template_hist_ws_size(int64_t ndocs);
int krca_template_hist(const uint64_t* hash, const int32_t* doc_lines, const int64_t* doc_line0, int64_t ndocs,
                       void* workspace, uint64_t* out_hash, int32_t* out_count, int32_t* n_templates, void* stream);
int32_t krca_template_max_lines(void);
/* containers with more than krca_template_max_lines() lines, one call each: the same output for
 * the container's n_lines hashes (hash, out_hash, out_count already offset to its doc_line0),
 * *n_templates set on the device; exact via a distinct-hash table + bucketed LDS sorts.
 * workspace: krca_template_huge_ws_size(n_lines) bytes, 16-byte aligned; *flag (device int32) = 1
 * if a bucket overflowed (then the output is incomplete and the caller must fail). */
int64_t krca_template_huge_ws_size(int64_t n_lines);
int krca_template_hist_huge(const uint64_t* hash, int64_t n_lines, void* workspace, uint64_t* out_hash,
                            int32_t* out_count, int32_t* n_templates, int32_t* flag, void* stream);

/* ---- a9: cross-pod Pearson correlation with per-pod top-k (new primitive; the
 * reference's only "correlation" is the string group-by of ref:agents/coordinator.py:118-155).
 * r(p,q) = Pearson over the T samples of metric channel `channel` of x[T][P][M] (population
 * std; a flat series correlates 0 with everything).  Per pod p: the k partners with the largest
 * |r| (self excluded, ties -> lower index) with r re-scored exactly (float64 over fp32 z), the
 * exact count of partners with |r| > tau (tau is float64, the type r is compared in: a float tau
 * of 0.6 would be 0.60000002 and miss pairs just above 0.6; the fp16 MFMA screening product decides every pair
 * farther than krca_corr_eps(T) from tau; the pairs within it are re-scored in float64: fails with
 * KRCA_EINVAL if more than 256*P + 2^20 pairs fall there, i.e. tau sits in the bulk of |r|), and
 * cert[p] > 0 iff the reported set is provably the exact top-k (pods whose first merge cannot
 * prove it have all their candidates re-scored; only a pod whose candidate buffer overflows twice
 * reports -1) (csrc/corr.hip).  Buffers: mean/scale [P]; z32 [P*T]; zh [krca_corr_pad_rows(P) *
 * krca_corr_pad_steps(T)] (fp16 bits); cand [krca_corr_cand_size(P, T, k) 4-byte words]; count [P];
 * out_idx/out_val [P*k]; cert [P].  k <= krca_corr_max_k(), 2 <= P <= 2^22.  krca_corr_topk
 * synchronises the stream once (it reads how many candidate buffers overflowed to decide on the
 * second pass).  The series must be finite: the certificates and the exact counts are proofs over
 * finite rows (a NaN row's products compare false everywhere; its results are unspecified).
 * Workspace size: cand holds the per-pod candidate buffers (8 KiB per pod), the threshold
 * sample's lists, the two ambiguous-pair lists of a main-pass batch (capped per batch), their
 * by-pod copy and the re-score's int16 partner rows (2 bytes per step per pod): at T = 1440,
 * k = 10 about 0.15 GB at 10k pods, 2.1 GB at 100k, 15.1 GB at 1M. */
int64_t krca_corr_pad_rows(int64_t P);
int32_t krca_corr_pad_steps(int32_t T);
int64_t krca_corr_cand_size(int64_t P, int32_t T, int32_t k);
int32_t krca_corr_max_k(void);
/* candidates buffered per pod by the main pass (cand's first [P][cap] int2 entries, then the [P] fill counts) */
int32_t krca_corr_cand_cap(void);
float krca_corr_eps(int32_t T);
int krca_corr_prepare(const float* x, int64_t P, int32_t M, int32_t T, int32_t channel, float* mean, float* scale,
                      float* z32, uint16_t* zh, void* stream);
int krca_corr_topk(const uint16_t* zh, const float* z32, int64_t P, int32_t T, int32_t k, double tau, void* cand,
                   int32_t* count, int32_t* out_idx, float* out_val, float* cert, void* stream);
/* a9 pod-sharded (kubernetes-rca-system_amd/krca/corr_dist.py): rank g of G owns pods
 * [lo, lo + n_loc), lo a multiple of 256; zh / z32 / phi are the all-gathered full arrays.  The
 * upper triangle is split by super-tile (every G-th from g); candidates travel to their pod's
 * owner in one all-to-all of int4 {pod, partner, r bits, 0} entries; count and raw_cnt [P] are
 * all-reduced (sum) by the caller.  ws: krca_corr_shard_ws_size(P, T, k, n_loc, G) 4-byte words. */
int64_t krca_corr_shard_ws_size(int64_t P, int32_t T, int32_t k, int64_t n_loc, int32_t G);
int krca_corr_shard_sample(const uint16_t* zh, int64_t P, int32_t T, int32_t k, int64_t lo, int64_t n_loc,
                           int32_t G, void* ws, float* phi, void* stream);
int krca_corr_shard_tiles(const uint16_t* zh, const float* z32, int64_t P, int32_t T, int32_t k, double tau, int32_t G,
                          int32_t g, const float* phi, int64_t n_loc, void* ws, int32_t* count, int32_t* raw_cnt,
                          void* stream);
int krca_corr_shard_pack_sizes(int64_t P, int32_t T, int32_t k, int64_t n_loc, int32_t G, int64_t n_max, void* ws,
                               int64_t* tot_host /*[G], synchronous*/, void* stream);
int krca_corr_shard_pack(int64_t P, int32_t T, int32_t k, int64_t n_loc, int32_t G, int64_t n_max, void* ws,
                         void* send, void* stream);
int krca_corr_shard_unpack(int64_t P, int32_t T, int32_t k, int64_t n_loc, int32_t G, int64_t lo, void* ws,
                           const void* recv, int64_t n_recv, void* stream);
int krca_corr_shard_merge(const uint16_t* zh, const float* z32, int64_t P, int32_t T, int32_t k, double tau,
                          int64_t lo, int64_t n_loc, int32_t G, const float* phi, int32_t* lcnt, void* ws,
                          int32_t* out_idx, float* out_val, float* cert, void* stream);

/* ---- a10: personalized PageRank root-cause propagation (replaces the sink of
 * Coordinator._identify_root_causes, ref:agents/coordinator.py:157-184; networkx 3.4.2
 * pagerank semantics: dangling mass follows the personalization, L1 stop rule err < N*tol,
 * tol <= 0 = exactly max_iter iterations).  Pull-CSR: row i lists the sources j of edges j->i;
 * outdeg[j] = out-degree of j.  Personalization p_i ∝ max(seed_i - seed_floor, 0) (uniform if
 * all are at the floor).  Arithmetic is 2^-60 fixed point in int64: results do not depend on
 * summation order or GPU count and are bit-identical to oracle/krca_oracle.c.  The per-node edge
 * weight floor(r_j * alpha / outdeg_j) travels as a 32-bit code (26 significant bits + shift,
 * truncating; csrc/ppr.hip wenc/wdec, restated in the oracle), so the gathered table is 4 B/node.
 * The codes bound the reachable tolerance: each sweep carries ~2^-26 of the mass in truncation, so
 * a tol below ~2^-26 / N (e.g. 1e-9 on a 2-node cycle) is not met -- krca_ppr then fails with
 * KRCA_ENOTCONV as the oracle reports no convergence (networkx would raise
 * PowerIterationFailedConvergence at its own, float64, limit).  networkx's default 1e-6 is met at
 * every N.
 * krca_ppr runs the whole iteration on one device (synchronous: returns *iters_host; since round
 * 3 with the folded steps below, one kernel per iteration); the
 * krca_ppr_shard_* steps are the same kernels for G pod-sharded ranks.  Per iteration:
 * krca_ppr_shard_step (pull SpMV fused with the rank update: gathers w_all, writes r_local and
 * this rank's send slice of krca_ppr_slice_words(n_max) int64 words: [n_max uint32 weight codes,
 * padded to 8 bytes | krca_ppr_nslot() int64 partial-sum slots]), then the host exchange (G > 1:
 * RCCL all-gather of send into w_all[G][slice]; G = 1: swap of two
 * buffers, no copy), then krca_ppr_shard_reduce (kubernetes-rca-system_amd/krca/rca.py).
 * ctl: krca_ppr_ctl_size(n_local) bytes, zero-filled by the caller once (long-row accumulators
 * live there and reset themselves). */
int32_t krca_ppr_nslot(void);
int64_t krca_ppr_slice_words(int64_t n_max); /* ceil(n_max / 2) + krca_ppr_nslot() */
int64_t krca_ppr_plan_size(const int64_t* row_ptr_host, int64_t N);
int krca_ppr_plan(const int64_t* row_ptr_host, int64_t N, int64_t* plan_host /*{rb,code,e0,e1} per block*/,
                  int64_t plan_len);
int64_t krca_ppr_workspace_size(int64_t N);
int krca_ppr(const int64_t* row_ptr, const int32_t* col /*pk*/, const int32_t* outdeg, int64_t N,
             const int64_t* plan, int64_t plan_len, const uint16_t* lane /*krca_ppr_pack*/, const float* seed,
             float seed_floor, double alpha, int32_t max_iter, double tol, void* workspace, float* r_out, int64_t* r_fixed /*nullable*/,
             int64_t* q_out /*nullable: quantised seeds*/, int32_t* iters_host, void* stream);
int64_t krca_ppr_ctl_size(int64_t n_local);
/* Host (no device work): the plan of krca_ppr_plan plus the packed column array pk_host[E]
 * (E = row_ptr_host[N]) the step kernel gathers through.  Columns are remapped to the exchange
 * layout in uint32 units (j + (j / n_max) * (2 * krca_ppr_slice_words(n_max) - n_max); n_max = N on
 * one device).  A short-row block whose distinct
 * columns are few enough becomes a DICTIONARY block: pk[e0, e0+nu) = its distinct columns
 * (ascending), then two uint16 slots per int32 word (16-byte aligned), one per edge; the plan
 * entry's first word carries nu in its high 32 bits (0 = direct block: pk[e] = column of edge e).
 * Each distinct column is gathered once per block instead of once per edge.  The DEVICE copy of
 * pk must have 64 zero words of padding past E (the step issues clamped 16-byte loads).  lane_host
 * [krca_ppr_lane_size(plan_len)] uint16: per block 2 x 256 words.  The block's non-empty rows get
 * consecutive sum slots 0, 1, ...; word t (lane t) = (slot of the row holding edge 8t) << 8 | the
 * bits of the edges 8t + 1 .. 8t + 7 that start a row, and word 256 + r = the slot of row rb + r
 * (256 for a row without edges), so the step's segmented row sums need neither a search nor the
 * row offsets.  Returns the number of dictionary blocks (>= 0) or a negative error (KRCA_EINVAL for a
 * column outside [0, N) or a remapped column id >= 2^30: the step addresses the gathered table at
 * 32-bit byte offsets).
 * (KRCA_PPR_DICT=0 packs every block direct; krca_ppr_remap_cols remaps a column array alone.) */
int64_t krca_ppr_lane_size(int64_t plan_len);
int64_t krca_ppr_pack(const int64_t* row_ptr_host, const int32_t* col_host, int64_t N, int64_t n_max,
                      int64_t* plan_host, int64_t plan_len, int32_t* pk_host, uint16_t* lane_host);
int krca_ppr_remap_cols(const int32_t* col, int64_t E, int64_t n_max, int32_t* out, void* stream);
/* p[0 .. n) = value by a kernel (not hipMemsetAsync): safe inside a HIP-graph capture whatever
 * the runtime's graph packet capture setting (the solve's zeroing uses kernels only) */
int krca_fill_i64(int64_t* p, int64_t n, int64_t value, void* stream);
/* Seeds are quantised to q = 2^32 per unit above seed_floor, clamped at 256 units (q <= 2^40; NaN
 * and values at or below the floor are 0), so the int64 seed total needs N <= 2^23 (KRCA_EINVAL
 * above). */
int krca_ppr_shard_init(const float* seed, float seed_floor, const int32_t* outdeg, int64_t n_local,
                        int64_t n_max, int64_t N, double alpha, void* ctl, int64_t* q_local,
                        int64_t* r_local, int64_t* send /*[krca_ppr_slice_words(n_max)]*/, void* stream);
int krca_ppr_shard_init_warm(const float* seed, float seed_floor, const int32_t* outdeg, int64_t n_local,
                             int64_t n_max, int64_t N, double alpha, void* ctl, int64_t* q_local,
                             const int64_t* r_local /*start vector: the previous solve*/, int64_t* send, void* stream);
/* flags of krca_ppr_shard_step: KRCA_PPR_RESIDUAL = accumulate |r_new - r_old| for the L1 stop
 * rule (reads r_local; needed when tol > 0), KRCA_PPR_WRITE_R = store r_new into r_local (every
 * iteration when tol > 0; a fixed-iteration solve needs it only on its last iteration). */
#define KRCA_PPR_RESIDUAL 1
#define KRCA_PPR_WRITE_R 2
int krca_ppr_shard_step(const int64_t* row_ptr, const int32_t* col /*pk*/, const int64_t* plan, int64_t plan_len,
                        const uint16_t* lane /*krca_ppr_pack*/, const int64_t* w_all /*[G][slice]*/, const int32_t* outdeg,
                        const int64_t* q_local, int64_t n_local, int64_t n_max, int64_t N, double alpha,
                        int32_t flags, int64_t* r_local, int64_t* send /*!= w_all*/, void* ctl, void* stream);
int krca_ppr_shard_reduce(const int64_t* w_all, int32_t G, int64_t n_max, int64_t N, double alpha,
                          double tol, int32_t first, void* ctl, int64_t* send_next, void* stream);
/* Folded iterations (the default of krca/rca.py): init (partial sums in slot set 0 of send; the
 * send slots and, at G = 1, the other buffer's must be zero before it), exchange, then per
 * iteration it = 1, 2, ...: krca_ppr_shard_step_folded + exchange, and krca_ppr_shard_finish(it =
 * the last) after the loop.  Step `it` does the reduction of step it - 1 itself (every workgroup
 * sums slot set (it - 1) % 3 of the G slices of w_all: convergence, teleport scale, iteration
 * count), adds its own partial sums into set it % 3 of send and zeroes set (it + 1) % 3 of
 * next_target, the buffer the NEXT step writes: at G = 1 the ping-pong buffer it gathers from
 * (w_all), at G > 1 the rank's send itself (the next step writes send again).  next_target is
 * send at G > 1; at G = 1 it is w_all when the exchange swaps the two buffers, or send when the
 * exchange copies send into w_all (a one-rank collective: krca.rca.Comm(collective=True)).  One
 * kernel and one exchange per iteration instead of two kernels; results bit-identical to the
 * unfolded sequence. */
int krca_ppr_shard_step_folded(const int64_t* row_ptr, const int32_t* col /*pk*/, const int64_t* plan, int64_t plan_len,
                               const uint16_t* lane, const int64_t* w_all, int32_t G, const int32_t* outdeg,
                               const int64_t* q_local, int64_t n_local, int64_t n_max, int64_t N, double alpha,
                               double tol, int32_t it, int32_t flags, int64_t* r_local, int64_t* send,
                               int64_t* next_target, void* ctl, void* stream);
int krca_ppr_shard_finish(const int64_t* w_all, int32_t G, int64_t n_max, int64_t N, double alpha, double tol,
                          int32_t it, void* ctl, void* stream);
/* Single device (G = 1, n_max = N): krca_ppr_shard_step with the iteration's krca_ppr_shard_reduce
 * (first = 0) done by the step's last workgroup — one launch per iteration instead of two.  Reads
 * the codes of w, writes r and send, zeroes w's partial-sum slots (w is the next step's write
 * target: the caller swaps w and send, exactly as around krca_ppr_shard_reduce). */
int krca_ppr_solo_step(const int64_t* row_ptr, const int32_t* col /*pk*/, const int64_t* plan, int64_t plan_len,
                       const uint16_t* lane, int64_t* w /*[slice(N)]*/, const int32_t* outdeg, const int64_t* q,
                       int64_t N, double alpha, int32_t flags, double tol, int64_t* r, int64_t* send /*!= w*/,
                       void* ctl, void* stream);
int krca_ppr_ctl_read(const void* ctl, int32_t* iters_host, int32_t* converged_host, void* stream);
/* the same two numbers without a synchronisation: enqueues their copy into host[0] = iteration at
 * convergence (0 = running), host[1] = iterations done; host should be pinned memory, read after
 * an event recorded behind it (the host's convergence polls then overlap the next iterations) */
int krca_ppr_ctl_copy(const void* ctl, int32_t* host /*[2]*/, void* stream);
int krca_ppr_fixed_to_float(const int64_t* r, int64_t n, float* out, void* stream);
/* root-cause key = bits of (double)r_i * (double)q_i: ranks pods by propagated mass times their
 * own anomaly; order-preserving as int64, fed to krca_topk_i64 (krca.rca.Config key "rq") */
int krca_ppr_rca_key(const int64_t* r, const int64_t* q, int64_t n, int64_t* key, void* stream);
/* The default root-cause key (krca.rca.Config key "explained"; the sink of
 * ref:agents/coordinator.py:157-184, edge direction of ref:agents/topology_agent.py:94-159: caller
 * -> dependency).  krca_rca_explain: over the WHOLE pull-CSR and the scores of every pod (score_all
 * [N]; q_j = the quantised seed of krca_ppr_shard_init), for each anomalous pod k A_k = its edges
 * from anomalous callers and S_k = the sum of their q; an anomalous dependency k of an anomalous pod
 * j (edge j -> k, j != k) explains j when (A_k - 1 >= A_j or q_k >= 2 q_j) and A_k q_j <= 3 S_k;
 * d_local[j - lo] = the largest q_k over the dependencies that explain j, for the pods [lo, hi) (0:
 * none).  Only anomalous pods' rows are walked; integer counts, sums and maxima, so bit-identical
 * to oracle/krca_oracle.c krco_rca_explain (S_k and A_k q_j in 128 bits: exact for any row).
 * ws: krca_rca_explain_ws_size(N) bytes, 16-byte aligned, no initialisation needed.
 * krca_rca_key_explained: key_i = bits(((double)recv_i + (double)t_i / 32) * (double)u_i) with u_i =
 * q_i - d_i (0 when <= 0), t_i the row's teleport share in the solve's last step (from the scale the
 * step recorded in ctl) and recv_i = r_i - t_i, the mass the row received from its callers: the rows
 * and ctl of a finished krca_ppr_shard_* / krca_ppr solve, N = the mesh's node count. */
int64_t krca_rca_explain_ws_size(int64_t N);
int krca_rca_explain(const float* score_all, int64_t N, float seed_floor, const int64_t* row_ptr, const int32_t* col,
                     int64_t lo, int64_t hi, int64_t* d_local /*[hi - lo]*/, void* ws, void* stream);
int krca_rca_key_explained(const int64_t* r_local, const int64_t* q_local, const int64_t* d_local, int64_t n_local,
                           int64_t N, const void* ctl, int64_t* key, void* stream);

/* ---- top-k (descending value, ties -> lower index), float32 or int64 keys; NaN keys are never
 * selected: with fewer than k non-NaN keys the remaining slots are idx -1, val -inf / INT64_MIN -- */
int64_t krca_topk_workspace_size(int64_t N, int32_t k);
int krca_topk_f32(const float* v, int64_t N, int32_t k, void* workspace, int32_t* idx, float* val,
                  void* stream);
int krca_topk_i64(const int64_t* v, int64_t N, int32_t k, void* workspace, int32_t* idx, int64_t* val,
                  void* stream);

/* ---- streaming rescoring (BASELINE configs[4]): krca_rolling_score carried
 * forward over a stream, delta new steps [delta][P][M] per call, global steps t0 .. t0+delta-1
 * (t0 == 0 starts the stream).  Outputs as krca_rolling_score over the whole series so far, with
 * n_exceed counted over the last H evaluated steps.  state: krca_stream_state_size bytes of plain
 * data (no pointers; set up by the t0 == 0 call): a copy to the host and back checkpoints the stream. */
int64_t krca_stream_state_size(int64_t P, int32_t M, int32_t W, int32_t H);
int krca_stream_score(const float* x_new, int64_t P, int32_t M, int32_t delta, int64_t t0, int32_t W, int32_t H,
                      float z_thr, void* state, float* z_last, float* score, int32_t* n_exceed, uint8_t* flags,
                      void* stream);

/* ---- f3: betweenness centrality for the SPOF check (TopologyAgent._analyze_single_points_of_failure,
 * ref:agents/topology_agent.py:322-356, networkx 3.4.2 betweenness_centrality): Brandes over the
 * OUT-edge CSR (row u = successors of u), `batch` sources in flight (one workgroup each),
 * float64, normalized / directed as networkx.  ws: krca_betweenness_ws_size(N, batch) bytes. */
int64_t krca_betweenness_ws_size(int64_t N, int32_t batch);
int krca_betweenness(const int64_t* row_ptr, const int32_t* col, int64_t N, int32_t normalized, int32_t directed,
                     int32_t batch, void* ws, double* bc, void* stream);

/* ---- f2: service-graph construction from Kubernetes objects (TopologyAgent._build_service_graph
 * ref:agents/topology_agent.py:94-160, _infer_dependencies_from_env :228-260; the same selector
 * test in ResourceAnalyzer._find_matching_pods ref:agents/resource_analyzer.py:835-854).
 * selector_match: bits[d * ceil(S/64) + s/64] bit s%64 = every item id of selector s occurs among
 *   the item ids of object d (ids interned by the host: krca/topograph.py); bit-exact.
 * substr_match: every (value v, key k) with key k occurring in value v (bytes), appended to
 *   out[cap] as v*K + k (once per occurrence, unordered); *n_out (device u64) = occurrences, may
 *   exceed cap.  lens = the distinct key lengths >= 1, ascending; table / hash from
 *   krca_substr_prepare (table_size = krca_substr_table_size(K) int32 slots). */
int krca_selector_match(const int32_t* lab, const int64_t* lab_off, int64_t D, const int32_t* sel,
                        const int64_t* sel_off, int64_t S, uint64_t* bits, void* stream);
int64_t krca_substr_table_size(int64_t K);
int krca_substr_prepare(const uint8_t* pat, const int64_t* pat_off, int64_t K, int32_t* table, int64_t table_size,
                        uint64_t* hash, void* stream);
int krca_substr_match(const uint8_t* text, const int64_t* val_off, int64_t V, const uint8_t* pat,
                      const int64_t* pat_off, int64_t K, const int32_t* table, int64_t table_size,
                      const uint64_t* hash, const int32_t* lens, int32_t n_lens, int64_t* out, int64_t cap,
                      uint64_t* n_out, void* stream);

/* ---- f1: pod status categorisation (ResourceAnalyzer._analyze_pods + _is_pod_healthy,
 * ref:agents/resource_analyzer.py:264-380, :856-895) over columnar pod status (encoding in
 * csrc/podstate.hip and krca/podstate.py): mask[p] bit b = membership of status group b in the
 * reference's dict order; hist[krca_pod_groups()] = group sizes.  Bit-exact. */
int32_t krca_pod_groups(void);
int krca_pod_classify(const uint8_t* pod_code, const int64_t* cont_off, const uint16_t* cont_code, int64_t P,
                      uint16_t* mask, int32_t* hist, void* stream);

/* ---- f4: group-bys of EventsAgent (ref:agents/events_agent.py:105-133 objects, :169-228 scheduling,
 * :230-290 volumes, :330-375 control plane, :377-446 nodes) and Coordinator._correlate_findings
 * (ref:agents/coordinator.py:118-155: group by component, max severity).  N membership records
 * (slot[i], key[i]); slots outside [0, S) are ignored; key < 0 = member that is not selected.
 * Output: one 8 x int64 record per slot, rec[s*8 + j]:
 *   j = 0      first member index (dict insertion order; INT32_MAX if the slot is empty)
 *   j = 1      (members << 32) | (members with key >= 0)
 *   j = 2 + r  r-th largest key >= 0 (-1 if none), r < R; ranks r >= 1 only over i < n_ranked.
 * Keys must be distinct within a slot for r >= 1 (the host packs (rank << 32) | (2^31-1-index)).
 * Bit-exact; 1 <= R <= krca_group_max_rank(), N < 2^31, 0 <= n_ranked <= N. */
int32_t krca_group_max_rank(void);
int krca_group_reduce(const int32_t* slot, const int64_t* key, int64_t N, int64_t n_ranked, int32_t S, int32_t R,
                      int64_t* rec, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KRCA_H */
