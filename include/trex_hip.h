/*
 * trex_hip.h -- C ABI of libtrexhip.so, the MI355X (gfx950) engine for trex's
 * batched Sankoff / tree-cost hot path.
 *
 * The reference (maraxen/trex) is pure Python/JAX with no FFI layer; its hot
 * path is a set of module functions.  Each entry point below replaces the
 * computation inside one of them (reference file:line cited per function);
 * the Python host (trex_amd/) keeps the reference's function names and
 * argument meaning and calls these through ctypes.  INTEGRATION.md shows the
 * binding a trex maintainer would add.
 *
 * Conventions
 *   - Every pointer passed to a trex_sankoff_* / trex_dp_* / trex_tree_* call
 *     is a DEVICE pointer owned by the caller, except where marked [host].
 *   - Calls are asynchronous on the caller's hipStream_t (`stream`, may be
 *     NULL = default stream); no allocation, no synchronisation, so a caller
 *     may capture them in a hipGraph.
 *   - Return 0 on success, a negative TREX_E_* code otherwise; the message of
 *     the last error on the calling thread is trex_last_error().
 *   - Node numbering is trex's: leaves 0..n_leaves-1, internal nodes
 *     n_leaves..n_all-1, root = n_all-1, n_leaves = (n_all+1)/2
 *     (src/trex/sankoff.py:46, src/trex/ground_truth.py:180-188).
 *   - Sites are the innermost (coalesced) axis of every per-site array.
 */
#ifndef TREX_HIP_H
#define TREX_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TREX_OK 0
#define TREX_E_ARG (-1)         /* bad argument / shape */
#define TREX_E_TOPOLOGY (-2)    /* topology the reference would hang on */
#define TREX_E_UNSUPPORTED (-3) /* valid input this build does not handle */
#define TREX_E_HIP (-4)         /* HIP runtime error */

/* flags for trex_sankoff_fwd / trex_sankoff_bwd */
#define TREX_FLAG_HARD_ROOT 1u  /* tau>0: site score = min(D_root), not smin */
/* 4 < Q <= 20 softmin: the lane-per-site kernel decides on the device, from
 * the cost matrix, whether it takes a call (a gate in the state-parallel
 * launch writes K, K^T and a flag into the workspace tail on every call).
 * Flag bit 2 (v8's TREX_FLAG_SITE_REUSE, which skipped that gate) is gone
 * since v9 and refused with TREX_E_ARG: it saved no measurable time and
 * trusted the caller to know when the cost changed. */

/* plan layout constants (see trex_plan_build).  A plan holds, after the
 * header, the forward steps [B][n_int][4], the backtrack entries
 * [B][n_int][2] and the staged (multi-wave) program of every tree (the
 * small-grid kernel, sankoff_staged.hip); trex_plan_ints sizes all of it. */
#define TREX_PLAN_HEADER_INTS 16

const char* trex_last_error(void);
/* ABI / plan-layout version.
 * 10: trex_dp_root_total (run_sankoff for Q > 128 on the raw-table path).
 * 9: TREX_FLAG_SITE_REUSE and trex_site_flag_offset removed (flags other
 *    than TREX_FLAG_HARD_ROOT are refused).
 * 8: plan child descriptors may carry bit 28 and step words flag 8 (deferred
 *    cherry edges of the Q <= 4 adjoint; plans are passed through unchanged,
 *    so bindings are unaffected); trex_tree_surrogate_constraint and
 *    trex_tree_update_tree_bwd_adam (fewer launches per C5 step).
 * 7: graph-capturable optimiser steps (device step state, *_dev entry
 *    points, trex_gumbel_noise); trex_tree_mf_rows_x3_codes takes the codes
 *    buffer size and Q.
 * 6: plans carry each tree's lane programs (the lane-per-site kernel for
 *    4 < Q <= 20, sankoff_site.hip) after the staged regions -- re-query
 *    trex_plan_ints; info[0] of trex_plan_build, the n_slots argument of
 *    trex_sankoff_fwd / _bwd / _fwd_bwd, is a packed word: the LDS stack
 *    depth | (lane-program slots + 1) << 16 (pass it through unchanged).
 * 5: plans carry each tree's staged (multi-wave) program after the
 *    backtrack entries (trex_plan_ints grew; a binding that sized or cached
 *    v4 plans must re-query it), Q up to 64, ragged Q > 4.
 * 4: site-major DP tables. */
int trex_version(void);

/* ------------------------------------------------------------------------
 * Topology plan (host side; topology is static per call like trex's jit
 * static args, src/trex/sankoff.py:114).
 *
 * children [host] int32 [B][n_all][2]: for every node the first two rows i
 *   with adjacency[i, node] == 1, filled with -1 -- exactly
 *   jnp.where(adjacency_matrix[:, node] == 1, size=2, fill_value=-1)
 *   (src/trex/sankoff.py:60) after run_sankoff zeroes adjacency[-1,-1]
 *   (sankoff.py:141).  Rows < n_leaves are ignored.
 * plan [host] int32 buffer of trex_plan_ints(B, n_all) ints; copy it to the
 *   device unchanged before the trex_sankoff_* calls.
 * info [host] int32[4] out: {n_slots, backtrack_ok, n_dag_nodes, n_unreached}
 *   n_slots = the packed slot word the kernels need (pass it unchanged to
 *   every call): bits 0-15 the LDS stack depth of the one-wave kernels,
 *   bits 16-31 the lane-per-site kernel's slot count + 1 (0: no lane
 *   programs fit);
 *   backtrack_ok = 0 when the reference's backtrack would not terminate
 *   (cyclic child references, sankoff.py:212-265); pass it on to
 *   trex_sankoff_backtrack, which then refuses with TREX_E_TOPOLOGY.
 * ---------------------------------------------------------------------- */
int64_t trex_plan_ints(int B, int n_all);
int trex_plan_build(const int32_t* children, int B, int n_all, int32_t* plan,
                    int32_t* info);

/* Workspace (device bytes) fwd/bwd/fwd_bwd use for a given shape: the
 * per-work-item fp64 partials (tree score, Q*Q dC) that a fixed-order reduce
 * kernel sums (bitwise reproducible), and for 4 < Q <= 64 the lane-per-site
 * kernel's gate words, K / K^T and cherry tables.  For 4 < Q <= 20 the value
 * also covers a region the size of the DP table (B * n_int * L * Q * 4 bytes)
 * where the fused call keeps its forward's softmin row sums for its adjoint;
 * a smaller workspace, down to the value minus B * n_int * L * Q * 4 bytes,
 * is accepted and the fused kernel then recomputes those sums (bitwise the
 * same results).  Zero it once with
 * trex_workspace_init before first use. */
int64_t trex_workspace_bytes(int B, int L, int n_all, int Q);
int trex_workspace_init(void* workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Forward DP.  Replaces vectorized_dp/run_dp + the total of run_sankoff
 * (src/trex/sankoff.py:24-97, 150-160, 187) for a batch of B trees.
 *   leaves   int8  [B][n_leaves][L]  state code in [0,Q); any other value is a
 *            leaf whose DP row stays all-1e5 (the reference's dropped scatter,
 *            sankoff.py:50)
 *   cost     fp32  [Q][Q]            substitution cost C[parent][child]
 *   tau      0 => hard min-plus (trex); >0 => softmin relaxation
 *   dp       fp32  internal rows (required), site-major [B][n_int][L][Q]
 *            (the reference's per-site (n_all, Q) rows without the leaf
 *            rows; a lane's Q states are one 8/12/16-byte access for Q <= 4,
 *            a lane group's row for the lane-per-state kernels, Q > 4)
 *   site_score fp32 [B][L] or NULL;  tree_score fp32 [B] (required)
 * Q up to 128 (leaf codes and ancestral states are int8): Q <= 64 on the
 * state-parallel / lane-per-site kernels, 64 < Q <= 128 on the large-alphabet
 * kernel (sankoff_bigq.hip, since ABI v7); Q > 128 returns
 * TREX_E_UNSUPPORTED (trex_amd.run_sankoff then takes the raw-table path:
 * trex_run_dp, trex_backtrack_generic, trex_dp_root_total).  Ragged batches
 * take the same range.
 * ---------------------------------------------------------------------- */
int trex_sankoff_fwd(const int32_t* plan, int n_slots, const int8_t* leaves,
                     const float* cost, int B, int L, int n_all, int Q, float tau,
                     unsigned flags, float* dp, float* site_score,
                     float* tree_score, void* workspace, int64_t workspace_bytes,
                     void* stream);

/* ------------------------------------------------------------------------
 * Adjoint (pre-order) sweep: gradient of sum_b d_tree_score[b]*tree_score[b]
 * w.r.t. the cost matrix -- what jax.grad of run_sankoff's total
 * (sankoff.py:187) w.r.t. cost_matrix computes for tau=0 (tie-averaged min
 * subgradient), and the softmin adjoint for tau>0.
 *   dp         fp32 DP table from trex_sankoff_fwd (same tau, same layout)
 *   d_tree_score fp32 [B] or NULL (= all ones)
 *   d_cost     fp32 [Q][Q] out (summed over trees, deterministic)
 *   marginals  fp32, dp's layout, or NULL: dScore/dD_v (soft ancestral
 *              state posteriors for tau>0)
 *   anc_states int8 [B][n_int][L] or NULL: argmax_i marginals (first index)
 * ---------------------------------------------------------------------- */
int trex_sankoff_bwd(const int32_t* plan, int n_slots, const int8_t* leaves,
                     const float* cost, int B, int L, int n_all, int Q, float tau,
                     unsigned flags, const float* dp, const float* d_tree_score,
                     float* d_cost, float* marginals, int8_t* anc_states,
                     void* workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Fused forward + adjoint in one launch (the benchmark step): writes dp,
 * tree_score (and site_score / marginals / anc_states when non-NULL) and
 * d_cost; each wave's adjoint re-reads the DP rows it has just written.
 * Same arguments and semantics as trex_sankoff_fwd followed by
 * trex_sankoff_bwd.
 * ---------------------------------------------------------------------- */
int trex_sankoff_fwd_bwd(const int32_t* plan, int n_slots, const int8_t* leaves,
                         const float* cost, int B, int L, int n_all, int Q, float tau,
                         unsigned flags, float* dp, float* site_score,
                         float* tree_score, const float* d_tree_score, float* d_cost,
                         float* marginals, int8_t* anc_states, void* workspace,
                         int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Ancestral reconstruction, bit-exact with the reference's backtrack:
 * root state = first argmin of dp[root] (sankoff.py:172), then the
 * reference's DFS (backtrack_sankoff_jit, sankoff.py:191-267) re-deriving
 * each child's state as the first argmin of C[s_parent] + D_child
 * (sankoff.py:67-69) instead of storing the backtracking table.
 *   dp         fp32 DP table from a tau=0 forward
 *   anc_states int8 [B][n_int][L] out (0 for nodes the DFS never reaches)
 * ---------------------------------------------------------------------- */
int trex_sankoff_backtrack(const int32_t* plan, int backtrack_ok, const float* cost,
                           const float* dp, int B, int L, int n_all, int Q,
                           int8_t* anc_states, void* stream);

/* ------------------------------------------------------------------------
 * Layout adapter to the reference's VmappedDPTable (L, n_all, Q)
 * (src/trex/utils/types.py:53, returned by run_sankoff sankoff.py:188):
 *   out fp32 [B][L][n_all][Q]; leaf rows synthesised from the codes
 *   (0 at the state, 1e5 elsewhere, sankoff.py:49-52,152).
 * ---------------------------------------------------------------------- */
int trex_dp_to_trex_layout(const float* dp, const int8_t* leaves, int B, int L,
                           int n_all, int Q, float* out, void* stream);

/* ------------------------------------------------------------------------
 * Raw-table entry points: the reference's own run_dp / vectorized_dp and
 * backtrack_sankoff_jit on its own table layouts, for callers that hold the
 * tables (src/trex/sankoff.py:24-97, 191-267; the reference's
 * tests/test_sankoff.py:31 calls run_dp with a caller-initialised table).
 * Exact reference semantics including caller-visible quirks (see rundp.hip):
 * leaf rows keep the caller's values except dp[i, int(seq)] = 0; nodes in
 * index order; child -1 reads the last row; not-yet-written rows hold the
 * caller's values; first argmin; jnp NaN rules.  Any Q.
 *   children  int32 [n_all][2], device: the first two rows with
 *             adjacency[row, node] == 1, -1 filled (sankoff.py:60; run_dp does
 *             NOT zero adjacency[-1, -1] -- run_sankoff does, :141)
 *   seqs      fp32 [n_seq >= (n_all+1)/2][n_codes][L] leaf states (vmapped
 *             run_dp: n_codes = 1, i.e. the (n, L) sequences; the unmapped
 *             run_dp with a (n, k) sequence array zeroes k states per leaf)
 *   dp        fp32 [L][n_all][Q] in/out (VmappedDPTable, utils/types.py:53)
 *   bt        fp32 [L][n_all][Q][4] in/out (BacktrackingTable, :56)
 * ---------------------------------------------------------------------- */
int trex_run_dp(const int32_t* children, int n_all, int L, int Q, const float* seqs,
                int n_codes, const float* cost, float* dp, float* bt, void* stream);

/* vmap(backtrack_sankoff_jit) over L sites (sankoff.py:166-180, 191-267):
 *   root_state int32 [L], or NULL: jnp.argmin(dp[:, root_node, :], axis=1)
 *   read from dp fp32 [L][n_all][Q] (sankoff.py:172; dp may be NULL when
 *   root_state is given); bt fp32 [L][n_all][Q][4]; out int32 [n_all][L]
 *   (the reference's out_axes=1); stack_ws >= trex_backtrack_workspace_bytes
 *   device bytes; status int32 [1] device, OR-ed with 1 when some site's DFS
 *   did not finish within max_steps pops (the reference would not terminate:
 *   a cyclic table).  The caller reads status after the stream completes. */
int64_t trex_backtrack_workspace_bytes(int n_all, int L);
int trex_backtrack_generic(int root_node, const int32_t* root_state, const float* dp,
                           const float* bt, int n_all, int n_leaves, int L, int Q, int32_t* out,
                           void* stack_ws, int64_t stack_bytes, int64_t max_steps, int32_t* status,
                           void* stream);

/* run_sankoff's total on a raw (L, n_all, Q) table (sankoff.py:187:
 * dp[:, -1].min(axis=1).sum(), NaN propagating): per-site root minima into
 * site_min fp32 [L] (scratch), their fp64 sum in a fixed order rounded to
 * fp32 into *total.  run_sankoff's path for Q > 128 (the raw run_dp table,
 * then this; trex_amd.run_sankoff), since ABI v10. */
int trex_dp_root_total(const float* dp, int L, int n_all, int Q, float* site_min, float* total,
                       void* stream);

/* 1 when the DP / marginal tables for Q states are site-major
 * [B][n_int][L][Q], 0 when they are [B][n_int][Q][L].  Always 1 since
 * trex_version() 4 (kept so bindings written against v3 still work). */
int trex_dp_site_major(int Q);

/* ========================================================================
 * Tree-cost path (src/trex/tree.py).  N = n_nodes, S = soft sequences
 * [N][L][Q] (flattened K = L*Q per node), A = adjacency [N][N] with
 * A[i][j] = "i is a child of j" (src/trex/utils/types.py:30-35).
 * ====================================================================== */

/* discretize_tree_topology (tree.py:31-47): out[i] = one_hot(argmax A[i]) */
int trex_tree_discretize(const float* A, int nrows, int ncols, int n_nodes, float* out,
                         void* stream);

/* update_seq (tree.py:110-130): S_anc[a][l] = softmax_q(T * X[a][l][q]),
 * written into rows n_leaf.. of S; and its VJP (dX = T S (dS - <S, dS>)). */
int trex_tree_update_seq(const float* x, int n_anc, int L, int Q, float temperature,
                         float* s_anc, void* stream);
int trex_tree_update_seq_bwd(const float* s_anc, const float* ds_anc, int n_anc, int L, int Q,
                             float temperature, float* dx, void* stream);

/* update_tree (tree.py:50-107) with explicit Gumbel noise (the reference's
 * jax.random.gumbel draw, :71): theta/noise/gates [N-1][n_anc] (noise,
 * gates may be NULL); A [N][N] = row softmax of the masked logits; VJP. */
int trex_tree_update_tree(const float* theta, const float* noise, const float* gates, int N,
                          int n_anc, float temperature, float* A, void* stream);
int trex_tree_update_tree_bwd(const float* A, const float* dA, const float* gates, int N,
                              int n_anc, float temperature, float* dtheta, void* stream);

/* Device workspace for the cost kernels below (split-K Gram partials etc.). */
int64_t trex_tree_workspace_bytes(int N, int64_t K);

/* compute_surrogate_cost (tree.py:163-209): loss[0] and, when non-NULL,
 * dS [N][K] = (diag(r+c) - (A+A^T)) S, dA [N][N] = (E_i+E_j)/2 - G_ij,
 * G_out [N][N] = S S^T.  Gram and dS run on f32 MFMA. */
int trex_tree_surrogate(const float* S, const float* A, int N, int64_t K, float* loss,
                        float* dS, float* dA, float* G_out, void* workspace,
                        int64_t workspace_bytes, void* stream);

/* The surrogate in phases (site-sharded data parallelism all-reduces the
 * N x N Gram matrix between the first two):  G = S S^T;  loss / dA / M =
 * diag(r+c) - (A+A^T) from (A, G);  dS = M S.  Workspace for combine: >= 8*N B. */
int trex_tree_gram(const float* S, int N, int64_t K, float* G, void* workspace,
                   int64_t workspace_bytes, void* stream);
/* As trex_tree_gram, but leaves G[i][j] untouched where both i and j lie in
 * the first floor(skip_rows/64)*64 rows: a cached constant block, e.g. the
 * fixed leaf x leaf Gram of the optimisation loop (leaf rows of S are data,
 * tree.py:127 rewrites only the ancestor rows). */
int trex_tree_gram_skip(const float* S, int N, int64_t K, int skip_rows, float* G,
                        void* workspace, int64_t workspace_bytes, void* stream);
/* Site-sharded optimisation with the cached leaf block: each rank's skip
 * Gram covers rows [row0, N) x all columns (row0 = floor(skip_rows/64)*64);
 * the ranks all-reduce those rows only (contiguous, row-major), then
 * G[i][j] = G[j][i] for i < row0 <= j restores the leaf rows' ancestor
 * columns from the reduced values (trex_amd.tree.TreeOptimizer(group=...)). */
int trex_tree_gram_mirror(float* G, int N, int row0, void* stream);
int trex_tree_surrogate_combine(const float* A, const float* G, int N, float* loss, float* dA,
                                float* M, void* workspace, void* stream);
int trex_tree_mf(const float* M, const float* S, int N, int64_t K, float* dS, void* stream);
/* dS rows [row0, row0 + nrows) only (dS_rows [nrows][K]): the optimiser needs
 * d loss / dS for the ancestor rows alone (leaf sequences are fixed,
 * tree.py:127), which halves the MF GEMM at N = 2 n_leaf - 1. */
int trex_tree_mf_rows(const float* M, const float* S, int N, int64_t K, int row0, int nrows,
                      float* dS_rows, void* stream);
/* f16x3 split-product versions of trex_tree_gram_skip / trex_tree_mf_rows:
 * each operand x is scaled by a power of two and split into f16 hi + lo
 * (22 significant bits), products hi*hi + hi*lo + lo*hi on f16 MFMA with f32
 * accumulation -- ~5x fewer MFMA cycles than the f32 MFMA, accuracy within
 * the same 1e-5 relative bar vs fp64 (tests/test_tree_gpu.py).  Contract:
 * every |operand| <= its max_abs (the optimisation loop's S is a softmax /
 * one-hot, max 1; M = diag(r+c) - (A+A^T) with softmax rows of A, max N+1);
 * a larger value overflows f16 (inf).  K % 4 == 0 (16-B aligned rows; a
 * ragged last 16- / 32-column block is masked), else TREX_E_UNSUPPORTED. */
int trex_tree_gram_skip_x3(const float* S, int N, int64_t K, int skip_rows, float max_abs,
                           float* G, void* workspace, int64_t workspace_bytes, void* stream);
int trex_tree_mf_rows_x3(const float* M, const float* S, int N, int64_t K, int row0, int nrows,
                         float max_abs_m, float max_abs_s, float* dS_rows, void* stream);
/* Leaf-code operand for the MF (Q = 4).  The leaf rows of S are fixed
 * one-hot data (trex's update_seq keeps sequences[:n_leaves],
 * tree.py:127-130), so dS = M S can read their codes instead of the f32 rows:
 * rows [0, lcr), lcr = trex_tree_leaf_code_rows(n_leaf) = 32 floor(n_leaf / 32),
 * are encoded once by trex_tree_leaf_codes into `codes` ([lcr][L] bytes,
 * trex_tree_leaf_codes_bytes).  *status (device int) is set to 1 when a row is
 * not exactly one-hot (the codes must then not be used).
 * trex_tree_mf_rows_x3_codes returns bitwise the result of trex_tree_mf_rows_x3
 * (one-hot x scale is exact in f16; the codes expand into the same split
 * planes) with a quarter of the operand bytes for those rows. */
int trex_tree_leaf_code_rows(int n_leaf);
int64_t trex_tree_leaf_codes_bytes(int n_leaf, int L);
int trex_tree_leaf_codes(const float* S, int n_leaf, int L, int Q, void* codes,
                         int64_t codes_bytes, int* status, void* stream);
int trex_tree_mf_rows_x3_codes(const float* M, const float* S, int N, int64_t K, int row0,
                               int nrows, float max_abs_m, float max_abs_s, const void* codes,
                               int64_t codes_bytes, int n_leaf, int Q, float* dS_rows,
                               void* stream);
/* (codes_bytes: the size of `codes`, >= trex_tree_leaf_codes_bytes(n_leaf, K / Q);
 * Q must be 4 and K = L * Q -- TREX_E_ARG otherwise, never a silent misread.) */

/* One C5 step's middle and tail in fewer launches (bitwise the separate
 * calls): trex_tree_surrogate_constraint = trex_tree_surrogate_combine then
 * trex_tree_constraint[_dev] with accumulate = 1 (state non-NULL: grad_scale
 * from the device step state's temperature; workspace holds N + (N-1)/2
 * doubles of partials); trex_tree_update_tree_bwd_adam =
 * trex_tree_update_tree_bwd then trex_adam_step[_dev] on the tree_params
 * (no clipping; dtheta may be NULL; state non-NULL: bias corrections from it,
 * count ignored).  tree.py:133-160 / 50-107 and optax adam.  M16 (optional):
 * M also written pre-split for trex_tree_mf_rows_x3p (below), ldm16 >= N
 * f32-equivalent columns per row, zero past N. */
int trex_tree_surrogate_constraint(const float* A, const float* G, int N, float scale,
                                   float grad_scale, const void* state, float* loss, float* dA,
                                   float* M, float max_abs_m, void* M16, int ldm16,
                                   void* workspace, void* stream);
int trex_tree_update_tree_bwd_adam(const float* A, const float* dA, const float* gates, int N,
                                   int n_anc, float T, float* dtheta, float* params, float* mu,
                                   float* nu, int count, const void* state, float lr, float b1,
                                   float b2, float eps, void* stream);

/* Pre-split f16x3 operands ("x3p").  The x3 GEMMs split every f32 operand
 * x * s (s = 2^(14 - ceil(log2 max_abs))) into f16 hi + lo each time they
 * stage it.  trex_tree_split_x3 stores that split once: every group of 4
 * consecutive values becomes 16 bytes (4 f16 hi, then 4 f16 lo), rows of ldo
 * f32-equivalent columns (ldo % 4 == 0, groups past cols zero), so the
 * pre-split operand has the f32 operand's byte offsets.  The x3p GEMMs read
 * it without the split arithmetic and give bitwise the x3 results:
 * trex_tree_gram_skip_x3p(S16, ...) == trex_tree_gram_skip_x3(S, ...);
 * trex_tree_mf_rows_x3p(M16, ldm, S16, ...) == trex_tree_mf_rows_x3[_codes]
 * (M16 rows ldm apart, ldm % 32 == 0, zero past N; codes optional);
 * trex_adam_seq_update_step_x3p == trex_adam_seq_update_step[_dev] (state
 * NULL: count / temperatures from the arguments) writing the next S rows
 * pre-split into s16_next (Q = 4, 16-B aligned). */
int trex_tree_split_x3(const float* X, int rows, int cols, int ldx, float max_abs, void* out,
                       int ldo, void* stream);
int trex_tree_gram_skip_x3p(const void* S16, int N, int64_t K, int skip_rows, float max_abs,
                            float* G, void* workspace, int64_t workspace_bytes, void* stream);
/* trex_tree_gram_skip_x3p_codes: the same Gram with rows [0, 32 (n_leaf / 32))
 * declared exact one-hot by their codes (the buffer trex_tree_leaf_codes
 * filled, status 0; Q = 4): their f16 lo plane is zero, so the lo x hi
 * products of those strips are skipped, and whole 128-row passes of them
 * are read as their code bytes instead of S16's 16-B pieces -- bitwise
 * trex_tree_gram_skip_x3p (S16's code rows must hold exactly the split of
 * the one-hot rows at this max_abs).  tree.py:199-209 (the surrogate's
 * S S^T).  Round 6. */
int trex_tree_gram_skip_x3p_codes(const void* S16, int N, int64_t K, int skip_rows, float max_abs,
                                  const void* codes, int64_t codes_bytes, int n_leaf, int Q,
                                  float* G, void* workspace, int64_t workspace_bytes,
                                  void* stream);
int trex_tree_mf_rows_x3p(const void* M16, int ldm, const void* S16, int N, int64_t K, int row0,
                          int nrows, float max_abs_m, float max_abs_s, const void* codes,
                          int64_t codes_bytes, int n_leaf, int Q, float* dS_rows, void* stream);
int trex_adam_seq_update_step_x3p(const float* ds_anc, int n_anc, int L, int Q, float temperature,
                                  float next_temperature, float* params, float* mu, float* nu,
                                  int count, float lr, float b1, float b2, float eps,
                                  const void* state, float max_abs_s, void* s16_next,
                                  void* stream);

/* compute_soft_cost (tree.py:212-266): ckind 0 = no C, 1 = C[Q] diagonal,
 * 2 = C[Q][Q]; W_scratch [N][L][Q] needed when ckind > 0. */
int trex_tree_soft_cost(const float* S, const float* A, const float* C, int ckind, int N, int L,
                        int Q, float* loss, float* W_scratch, void* workspace,
                        int64_t workspace_bytes, void* stream);

/* enforce_graph_constraints (tree.py:133-160): loss = [loss +]
 * grad_scale * scale * sum_cols (colsum - 2)^2; dA (optional) +=
 * grad_scale * 2 scale (colsum - 2) on the constrained block. */
int trex_tree_constraint(const float* A, int N, float scale, float grad_scale, float* loss,
                         int accumulate, float* dA, void* workspace, void* stream);

/* compute_cost (tree.py:269-296): exact cost of a labelled tree. */
int trex_tree_compute_cost(const float* S, const float* A, const float* subst, int N, int L,
                           int Q, float* cost, void* workspace, void* stream);

/* optax adam (b1, b2, eps, eps_root = 0) fused update of one tensor, step
 * `count` (1-based); optional clip_by_global_norm(clip_norm) using squared
 * norm partials from trex_sq_norm_parts over ALL gradient tensors. */
int trex_adam_step(float* params, const float* grads, float* mu, float* nu, int64_t n,
                   int count, float lr, float b1, float b2, float eps,
                   const double* grad_sq_norm_parts, int n_parts, float clip_norm,
                   void* stream);
int trex_sq_norm_parts(const float* x, int64_t n, double* parts, int n_parts, void* stream);
/* The optimisers of create_optimizer (src/trex/evals/benchmark.py:41-72),
 * optax 0.2.6 semantics, one tensor per call, optionally after
 * clip_by_global_norm (squared-norm partials of ALL gradient tensors):
 *   kind 0 adam(lr, b1, b2, eps)            state1 = mu, state2 = nu
 *   kind 1 adamw(lr, b1, b2, eps, wd)       state1 = mu, state2 = nu
 *   kind 2 sgd(lr, momentum = b1)           state1 = trace
 *   kind 3 rmsprop(lr, decay = b2, eps)     state2 = nu  (eps inside the sqrt)
 * count is the 1-based step (bias correction). */
int trex_optax_step(int kind, float* params, const float* grads, float* state1, float* state2,
                    int64_t n, int count, float lr, float b1, float b2, float eps,
                    float weight_decay, const double* grad_sq_norm_parts, int n_parts,
                    float clip_norm, void* stream);
/* update_seq's VJP (trex_tree_update_seq_bwd) fused into the Adam update of
 * the ancestor logits (no clipping): params / mu / nu [n_anc][L][Q] updated
 * in place from s_anc = softmax(T x) and ds_anc = d loss / d s_anc; the
 * logits gradient is written to grads_out only when non-NULL.  Bitwise the
 * same as trex_tree_update_seq_bwd followed by trex_adam_step. */
int trex_adam_seq_step(const float* s_anc, const float* ds_anc, int n_anc, int L, int Q,
                       float temperature, float* params, float* mu, float* nu, int count,
                       float lr, float b1, float b2, float eps, float* grads_out, void* stream);
/* trex_adam_seq_step with update_seq (src/trex/tree.py:110-130) folded in on
 * both sides, for a loop whose S rows come from this call: the step's
 * s_anc = softmax(temperature * params) is recomputed from params (bitwise
 * what trex_tree_update_seq wrote), and after the Adam update the next
 * step's rows softmax(next_temperature * params_new) are written to s_next
 * [n_anc][L][Q] (may be the S buffer the caller's GEMMs read this step). */
int trex_adam_seq_update_step(const float* ds_anc, int n_anc, int L, int Q, float temperature,
                              float next_temperature, float* params, float* mu, float* nu,
                              int count, float lr, float b1, float b2, float eps, float* s_next,
                              void* stream);

/* ------------------------------------------------------------------------
 * Graph-capturable optimisation loops (ABI v7).  The reference runs its
 * optimiser inside lax.fori_loop / lax.scan (src/trex/evals/benchmark.py:
 * 167-200; tests/test_convergence.py:238-261 jits the step), i.e. the step
 * count, the annealed temperature and the Gumbel key are device values.  Here
 * they live in a device "step state" (trex_step_state_bytes() bytes, zeroed
 * or holding the count of the steps already taken in its first int32):
 *   trex_step_advance: count += 1, then Adam's bias corrections
 *     1 - b^count (b1, b2; computed exactly as the host-count entry points
 *     do, so both give bitwise the same update) and, when temps [n_temps] is
 *     given (an annealing schedule on the device), this step's temperature
 *     T = temps[count - 1] and the next one's Tn = temps[count] (clamped to
 *     the last entry).  Launch it first in every step.
 *   *_dev: the entry points above with count / temperature read from the
 *     state instead of host arguments (trex_tree_constraint_dev: grad_scale =
 *     T; trex_adam_seq_update_step_dev: temperature = T, next = Tn).
 *   trex_gumbel_noise: Gumbel(0, 1) noise out f32 [n] for the state's step
 *     (state NULL: step 0), a pure function of (seed, step, index) -- the
 *     reference's per-step jax.random.gumbel(step_key) (tree.py:71);
 *     counter-based splitmix64 draws, restated in oracle/datagen_ref.py.
 * A step built from these launches only kernels whose arguments do not
 * change between steps, so it can be captured once in a hipGraph and
 * replayed (trex_amd.tree.TreeOptimizer.device_loop, trex_amd.tree.Adam). */
int trex_step_state_bytes(void);
int trex_step_advance(void* state, float b1, float b2, const float* temps, int64_t n_temps,
                      void* stream);
int trex_adam_step_dev(float* params, const float* grads, float* mu, float* nu, int64_t n,
                       const void* state, float lr, float b1, float b2, float eps,
                       const double* grad_sq_norm_parts, int n_parts, float clip_norm,
                       void* stream);
int trex_optax_step_dev(int kind, float* params, const float* grads, float* state1,
                        float* state2, int64_t n, const void* state, float lr, float b1, float b2,
                        float eps, float weight_decay, const double* grad_sq_norm_parts,
                        int n_parts, float clip_norm, void* stream);
int trex_adam_seq_update_step_dev(const float* ds_anc, int n_anc, int L, int Q, const void* state,
                                  float* params, float* mu, float* nu, float lr, float b1,
                                  float b2, float eps, float* s_next, void* stream);
int trex_tree_constraint_dev(const float* A, int N, float scale, const void* state, float* loss,
                             int accumulate, float* dA, void* workspace, void* stream);
int trex_gumbel_noise(uint64_t seed, const void* state, int64_t n, float* out, void* stream);

/* ========================================================================
 * Ragged batches: trees of different sizes (n_all_b taxa+ancestors) and
 * site counts (L_b) in ONE launch -- what trex gets from padding every tree
 * to MAX_NODES / N buckets with node and site masks (src/trex/padding.py:
 * 25-27, 77-297) so one jit serves mixed sizes, without the padded work.
 *   children  int32, tree b's [n_all_b][2] child lists concatenated
 *   plan      trex_ragged_plan_ints(B, n_all, L) ints; copy to the device
 *   info      int64 [8] out: n_slots, max_n_leaves, items (64-site work
 *             items), leaf bytes (sum n_leaves_b L_b), DP row-sites
 *             (sum n_int_b L_b), sites (sum L_b), backtrack_ok,
 *             dag | unreached << 32
 * Packed tensors: leaves int8 [sum n_leaves_b L_b] (tree b: [n_leaves_b][L_b]);
 * dp / marginals f32 [sum n_int_b L_b][Q] (tree b: [n_int_b][L_b][Q]);
 * site_score f32 [sum L_b]; anc_states int8 [sum n_int_b L_b];
 * tree_score / d_tree_score [B].  Q <= 128 (4 < Q <= 64: the
 * state-parallel kernel, each 64-site item split over ceil(64 /
 * sites-per-wave) waves; 64 < Q <= 128: the large-alphabet kernel, a
 * 128-thread workgroup per item; the workspace is sized by
 * trex_ragged_workspace_bytes(items, Q)).  phase: 1
 * forward, 2 adjoint, 3 fused (same semantics as trex_sankoff_fwd / _bwd /
 * _fwd_bwd per tree).
 * ---------------------------------------------------------------------- */
int64_t trex_ragged_plan_ints(int B, const int32_t* n_all, const int32_t* L);
int trex_ragged_plan_build(const int32_t* children, const int32_t* n_all, const int32_t* L, int B,
                           int32_t* plan, int64_t* info);
int64_t trex_ragged_workspace_bytes(int64_t items, int Q);
int trex_sankoff_ragged(int phase, const int32_t* plan, int B, int n_slots, int max_n_leaves,
                        int64_t items, const int8_t* leaves, const float* cost, int Q, float tau,
                        unsigned flags, float* dp, float* site_score, float* tree_score,
                        const float* d_tree_score, float* d_cost, float* marginals,
                        int8_t* anc_states, void* workspace, int64_t workspace_bytes,
                        void* stream);
/* trex-exact ancestral states per tree (backtrack_sankoff_jit) for a ragged
 * batch; steps = sum n_int_b (plan header int 2). */
int trex_sankoff_ragged_backtrack(const int32_t* plan, int B, int64_t items, int64_t steps,
                                  int backtrack_ok, const float* cost, const float* dp, int Q,
                                  int8_t* anc_states, void* stream);

/* ========================================================================
 * Synthetic data on the device: trex's
 * generate_groundtruth (src/trex/ground_truth.py:112-197, mutate :20-52) and
 * iid uniform leaf states, from a counter-based generator (splitmix64 of
 * (seed, stream, counter); trex's JAX threefry streams cannot be
 * reproduced, the process can).  Restated in oracle/datagen_ref.py.
 *   seqs int8 [2 n_leaves - 1][L] out: root (last row) zero, every child =
 *     its parent with exactly n_mutations distinct sites moved by
 *     1 + U{0..Q-2} (mod Q); balanced numbering (children of parent p are
 *     2(p - n_leaves), 2(p - n_leaves) + 1).  n_leaves a power of 2.
 *   workspace trex_datagen_workspace_bytes(n_leaves, n_mutations) bytes.
 * ---------------------------------------------------------------------- */
int64_t trex_datagen_workspace_bytes(int n_leaves, int n_mutations);
int trex_datagen_groundtruth(uint64_t seed, int n_leaves, int L, int Q, int n_mutations,
                             int8_t* seqs, void* workspace, int64_t workspace_bytes,
                             void* stream);
/* out int8 [n]: uniform states in [0, Q) */
int trex_datagen_uniform_states(uint64_t seed, int64_t n, int Q, int8_t* out, void* stream);
/* nk_model.generate_tree_data (src/trex/nk_model.py:116-278): NK-model
 * sequence evolution along a tree, branch_length Metropolis steps per edge
 * (coupled redraw of a site and its K interactions with probability
 * coupled_prob, else per-site Bernoulli(rate) redraws; rate =
 * min(mutation_rate exp(N(0,1) noise_std), 1) per edge; accepted with
 * probability min(1, exp(f_new - f_cur)), f = mean site fitness).  Same
 * counter-based draws as above (restated in oracle/datagen_ref.py).
 *   interactions int32 [L][K], fitness f32 [L][Q^(K+1)] (device)
 *   parent int32 [n_nodes] (device); order int32 [n_slots] (device): the
 *     reference's BFS sorted_nodes -- root first, then each level, and the
 *     node n_nodes - 1 repeated for every slot the BFS did not fill (its -1
 *     index, nk_model.py:186-190, 236-245; trex_amd.datagen.bfs_levels
 *     builds it); level_offsets int32 [n_levels + 1] (HOST array): slots
 *     [level_offsets[lv], level_offsets[lv + 1]) run in one launch, so each
 *     level's nodes must have their parents in earlier levels; slot s
 *     draws from streams 4s .. 4s + 3
 *   seqs int8 [n_nodes][L] in/out: the root row holds the root sequence;
 *     every other row is written.  L <= 65536, Q^(K+1) < 2^31. */
int trex_datagen_nk_tree(uint64_t seed, int n_nodes, int L, int Q, int K, const int* interactions,
                         const float* fitness, const int* parent, const int* order,
                         const int* level_offsets, int n_levels, float mutation_rate,
                         float noise_std, float coupled_prob, int branch_length, int8_t* seqs,
                         void* stream);

/* ========================================================================
 * NK landscape-aware loss (src/trex/evals/benchmark.py): the parental
 * guidance term of _compute_loss_landscape_aware_stacked (:235-306) on top
 * of the surrogate cost, with compute_parental_logits (:586-663).
 *   S            fp32 [N][L][Q]  soft sequences (after update_seq)
 *   interactions int32 [L][k]    epistatic partners, k = interactions.shape[1]
 *   fitness      fp32 [L][Q^(k+1)], index s * Q^k + sum_j c_j Q^(k-1-j)
 *                (the site's own state most significant, then neighbour 0:
 *                the reference's reshape(n_states, -1), :647)
 * Limits: Q <= 32, k <= 16, k * Q <= 128.
 * ---------------------------------------------------------------------- */

/* logits [R][L][Q] of parent rows rows[0..R) of S (compute_parental_logits;
 * k = 0 returns the (L, Q) table per row, :612-620). */
int trex_nk_parental_logits(const float* S, const int32_t* rows, int R, int L, int Q,
                            const int32_t* interactions, int k, const float* fitness,
                            float* logits, void* stream);

/* Host planner, once per (parent map, landscape): parent[n] = argmax_j
 * A[n][j] (benchmark.py:286, first index).  info[0] = number of distinct
 * parent rows (n_parents), info[1] = #nodes with parent != self (the
 * cross-entropy normaliser, :302). Copy the plan to the device. */
int64_t trex_nk_plan_ints(int N, int L, int k);
int trex_nk_plan_build(const int32_t* parent, int N, const int32_t* interactions, int L, int k,
                       int32_t* plan, int32_t* info);
int64_t trex_nk_workspace_bytes(int N, int L, int Q, int k, int n_parents);

/* loss = surrogate[0] + lambda * CE / (n_nonroot * n_valid) with CE the
 * masked cross-entropy of every node's sequence against log_softmax of its
 * parent's logits (:288-302).  seq_mask fp32 [L] (1 valid / 0) or NULL;
 * n_valid = sum(seq_mask) (L when NULL).  d_S (optional) [N][L][Q] =
 * d_S_in (optional: e.g. the surrogate's gradient) + d(lambda * fitness)/dS
 * through both the child and the parent role. */
int trex_nk_landscape_loss(const int32_t* plan, int n_parents, const float* S, int N, int L,
                           int Q, const int32_t* interactions, int k, const float* fitness,
                           const float* seq_mask, float n_valid, float lambda_val, int n_nonroot,
                           const float* surrogate, const float* d_S_in, float* loss, float* d_S,
                           void* workspace, int64_t workspace_bytes, void* stream);

/* ========================================================================
 * Multi-GPU exchange: the sharded paths' only collective
 * is the sum over ranks of one small fp32 buffer -- [dC, loss] (Q*Q + 1
 * floats) for the tree-batch-sharded Sankoff step, the N x N Gram for the
 * site-sharded tree-cost step.  One RCCL all-reduce on the caller's stream.
 * RCCL is loaded with dlopen on first use (TREX_E_UNSUPPORTED if absent).
 *   trex_comm_get_unique_id: on one rank; broadcast the bytes to the others
 *   trex_comm_init: one communicator per (process, device ordinal dev); the
 *     returned comm is an ncclComm_t -- a caller's own RCCL communicator may
 *     be passed to trex_allreduce_sum instead
 *   trex_allreduce_sum: buf [count] fp32 device, in place, summed over ranks
 * ---------------------------------------------------------------------- */
int trex_comm_unique_id_bytes(void);
int trex_comm_get_unique_id(void* id);
int trex_comm_init(void** comm, int nranks, const void* id, int rank, int dev);
int trex_comm_destroy(void* comm);
int trex_allreduce_sum(float* buf, int count, int dev, void* comm, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TREX_HIP_H */
