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

/* plan layout constants (see trex_plan_build) */
#define TREX_PLAN_HEADER_INTS 16

const char* trex_last_error(void);
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
 *   n_slots = LDS stack depth the kernels need (pass to every call);
 *   backtrack_ok = 0 when the reference's backtrack would not terminate
 *   (cyclic child references, sankoff.py:212-265); pass it on to
 *   trex_sankoff_backtrack, which then refuses with TREX_E_TOPOLOGY.
 * ---------------------------------------------------------------------- */
int64_t trex_plan_ints(int B, int n_all);
int trex_plan_build(const int32_t* children, int B, int n_all, int32_t* plan,
                    int32_t* info);

/* Workspace (device bytes) needed by fwd/bwd for a given shape.  It holds
 * per-block partial sums and arrival counters for the in-kernel,
 * fixed-order (bitwise reproducible) reductions; zero it once with
 * trex_workspace_init before first use (the kernels leave it zeroed). */
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
 *   dp       fp32  [B][n_int][Q][L]  internal rows (required)
 *   site_score fp32 [B][L] or NULL;  tree_score fp32 [B] (required)
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
 *   dp         fp32 [B][n_int][Q][L] from trex_sankoff_fwd (same tau)
 *   d_tree_score fp32 [B] or NULL (= all ones)
 *   d_cost     fp32 [Q][Q] out (summed over trees, deterministic)
 *   marginals  fp32 [B][n_int][Q][L] or NULL: dScore/dD_v (soft ancestral
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
 *   dp         fp32 [B][n_int][Q][L] from a tau=0 forward
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

#ifdef __cplusplus
}
#endif

#endif /* TREX_HIP_H */
