// Shared constants and error plumbing for libtrexhip.so (host side).
#pragma once

#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/trex_hip.h"

namespace trex {

constexpr int32_t kPlanMagic = 0x54524558;  // 'TREX'

// forward-step child descriptor: index bits 0-15, slot 16-23, kind 24-25
constexpr int32_t kStepAccumulate = 1 << 26;  // adjoint: add into the slot
// register bypass: this internal child is the previous step's node (its only
// consumer is this step): forward reads its D from registers, the adjoint
// hands its cotangent to the next reverse step in registers
constexpr int32_t kChildPrev = 1 << 27;
// deferred edge (Q <= 4 adjoint; other kernels ignore it): this internal
// child is a cherry (both of its children leaves / 1e5 rows) with one
// parent.  The parent's step hands its own cotangent to the child's slot
// (or the bypass) instead of the child's, reading no DP row; the child's step
// (kStepDeferredIn) recomputes its D from its leaf messages and runs the edge
// adjoint first.  A cherry's row is then never re-read from HBM.
constexpr int32_t kChildDeferred = 1 << 28;
// forward-step flags (word 3)
constexpr int32_t kStepRoot = 1;
constexpr int32_t kStepUnreached = 2;
constexpr int32_t kStepToNext = 4;  // output consumed only by the next step (bypass)
constexpr int32_t kStepDeferredIn = 8;  // slot / bypass holds the parent's cotangent

// Staged (multi-wave) program, after the backtrack entries of a plan: one
// region of staged_tree_ints(ni) ints per tree, steps [ni][4] (same words as
// the forward steps; every internal row has its own LDS slot = its row, so
// no slot / bypass fields) | S (stages) | offsets [S * kStageWaves + 1]:
// steps of stage s on wave w are [off[s*W + w], off[s*W + w + 1]).  The
// waves of one workgroup run a stage's node lists in parallel, a barrier
// between stages (sankoff_staged.hip).
constexpr int kStageWaves = 8;
inline int64_t staged_tree_ints(int ni) {
  return 4LL * ni + (((int64_t)ni * kStageWaves + 2 + 3) & ~3LL);
}

// Lane-per-site program (sankoff_site.hip), after the staged regions: one
// region of lp_tree_ints(ni) ints per tree (plan.cpp lane_program_one_tree):
//   [0] S (stages)  [1] n_slots (-1: the tree cannot run it)  [2] n_steps
//   [3] n_inline  [4 .. 4 + S] stage offsets: stage s = steps [off[s], off[s+1])
//   steps at lp_steps_offset(ni): [n_steps][4] = {row | slot << 16,
//     child desc 0, child desc 1, flags (kStepRoot)}, then the inline rows
//     [n_inline][4] = {row, child desc 0, child desc 1, height}, children first.
//   child desc: kind << 24 | (sentinel: 0; leaf: leaf index; task row:
//     row | slot << 16 (kKindInt); inline row: its index (kKindInline))
constexpr int kKindInline = 3;
inline int64_t lp_steps_offset(int ni) { return 8 + (((int64_t)ni + 1 + 3) & ~3LL); }
inline int64_t lp_tree_ints(int ni) { return lp_steps_offset(ni) + 4LL * ni; }

// backtrack entry kinds (bits 16-19 of word 0)
constexpr int kBtRoot = 0;
constexpr int kBtReal = 1;
constexpr int kBtSentinel = 2;
constexpr int kBtUnreached = 3;

int set_error(int code, const char* fmt, ...);

// Host argument checks on the IEEE bit pattern: the library is compiled with
// -fno-honor-nans (kernels drop NaN canonicalisation), under which the
// compiler may fold `!(x >= 0.0f)` or std::isnan(x) to false for a NaN x.
inline uint32_t float_bits(float x) {
  uint32_t u;
  std::memcpy(&u, &x, sizeof u);
  return u;
}
inline bool finite_f32(float x) { return (float_bits(x) & 0x7f800000u) != 0x7f800000u; }
// finite and >= 0 (-0.0 included)
inline bool nonneg_finite_f32(float x) {
  const uint32_t u = float_bits(x);
  return finite_f32(x) && (!(u >> 31) || (u & 0x7fffffffu) == 0);
}
// finite and > 0
inline bool pos_finite_f32(float x) {
  const uint32_t u = float_bits(x);
  return finite_f32(x) && !(u >> 31) && (u & 0x7fffffffu) != 0;
}

// ---- Q > 4: state-parallel kernels on a site-major DP table (sankoff_wide.hip)
struct WideCall {
  int phase;  // 1 fwd, 2 adjoint, 3 fused
  bool soft;
  const int* steps;
  const int8_t* leaves;
  const float* cost;
  int B, L, nl, ni, Q, n_slots;
  float a, bcoef;
  int hard_root;
  float* dp;
  float* site_score;
  float* tree_score;
  const float* dts;
  float* marg;
  int8_t* anc;
  float* d_cost;
  void* workspace;
  void* stream;
  // set when the lane-per-site kernel (sankoff_site.hip) ran first: the device
  // word it wrote (1: it handled the launch -- the state-parallel kernels
  // exit at once, the reduce sums its mx_tiles partials per tree)
  const int* mx_flag = nullptr;
  int mx_tiles = 0;
  // gated launch (run_phase): the state-parallel kernel decides per
  // workgroup whether the lane-per-site kernel takes the call and writes
  // its K / K^T (site_kg) and the flag (site_flag) from workgroup 0
  int* site_flag = nullptr;
  float* site_kg = nullptr;
  // fused site kernel: its forward's softmin row sums s = K u of every
  // internal child row it computes, re-read by its adjoint (workspace past
  // the wide workspace, DP-table layout; null: recomputed)
  float* site_srow = nullptr;
};
constexpr int kWideMaxQ = 64;
// 64 < Q <= 128: the large-alphabet kernel (sankoff_bigq.hip; int8 leaf codes
// and ancestral states bound Q by 128)
constexpr int kBigMaxQ = 128;
int bigq_tiles(int L);
int64_t bigq_workspace_bytes(int B, int L, int Q);
int bigq_run(const char* fn, const WideCall& c);
int bigq_backtrack(const int32_t* bt, const float* cost, const float* dp, int B, int L, int ni,
                   int Q, int8_t* anc, void* stream);
int bigq_ragged_run(const char* fn, const WideCall& c, const int* rmeta, const int* ritem,
                    int64_t items);
int bigq_ragged_backtrack(const int32_t* rmeta, int B, int64_t items, int64_t steps,
                          const float* cost, const float* dp, int Q, int8_t* anc, void* stream);
constexpr int kRaggedMeta = 12;  // ints per tree record of a ragged plan (plan.cpp)  // leaf codes and ancestral states are int8
int wide_group(int Q);
int wide_tiles(int L, int Q);
size_t wide_lds_bytes(int n_slots, int nl, int ni, int Q);
int64_t wide_workspace_bytes(int B, int L, int Q);
int wide_run(const char* fn, const WideCall& c, bool reduce = true);
// staged multi-wave kernel (sankoff_staged.hip); staged = the plan's staged
// regions (after the backtrack entries)
size_t staged_lds_bytes(int ni, int nl, int Q, int phase);
int staged_run(const char* fn, const WideCall& c, const int32_t* staged);
// fixed-order sum of per-item partials -> tree_score [B] (phase & 1), d_cost
// [Q*Q] (phase & 2); part_dc is [Q*Q][B*tiles]
// (ragged batches: first[b * first_stride] is tree b's first item, items the
// total; tiles is then unused)
// (first_scale: partials per item, the wide kernel's waves per ragged item)
// (mx_flag / mx_tiles: when *mx_flag is set on the device, the partials are
// the lane-per-site kernel's, mx_tiles per tree)
int partial_reduce(const char* fn, const double* part_tree, const double* part_dc, int B,
                   int tiles, int Q, int phase, float* tree_score, float* d_cost, void* stream,
                   const int* first = nullptr, int first_stride = 0, int items = 0,
                   int first_scale = 1, const int* mx_flag = nullptr, int mx_tiles = 0);
// ragged batches with Q > 4 on the wide kernel (rmeta / ritem: the plan's
// records and item table; c.nl = max leaves, c.L unused)
int64_t wide_ragged_workspace_bytes(int64_t items, int Q);
int wide_ragged_run(const char* fn, const WideCall& c, const int* rmeta, const int* ritem,
                    int64_t items);
// lane-per-site kernel for the factored softmin, 4 < Q <= 20 (sankoff_site.hip)
bool site_eligible(const WideCall& c, int lp_slots);
constexpr int kSiteMaxQ = 20;  // the lane-per-site kernel's largest Q (kSiteSQ, wide_dev.h)
bool site_srow_on();  // TREX_SITE_SROW != "0" (read per call)
inline int64_t site_srow_offset(int B, int L, int Q) {
  return (wide_workspace_bytes(B, L, Q) + 255) / 256 * 256;
}
int site_tiles(int L);
int site_run(const char* fn, const WideCall& c, const int32_t* lanes, int lp_slots,
             const int* flag, const float* kg);
// the same with each site's states split over a wave pair (sankoff_site2.hip;
// TREX_SITE2=1 / 8 / 6 / 4, read per call: the pair count, when its LDS fits)
bool site2_on(int lp_slots, int nl, int ni);
int site2_run(const char* fn, const WideCall& c, const int32_t* lanes, int lp_slots,
              const int* flag, const float* kg);
int wide_backtrack(const int32_t* bt, const float* cost, const float* dp, int B, int L, int ni,
                   int Q, int8_t* anc, void* stream);
int wide_ragged_backtrack(const int32_t* rmeta, int B, int64_t items, int64_t steps,
                          const float* cost, const float* dp, int Q, int8_t* anc, void* stream);

}  // namespace trex
