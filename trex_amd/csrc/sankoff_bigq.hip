// libtrexhip.so -- Sankoff for large alphabets, 64 < Q <= 128 states (gfx950).
//
// trex sizes every table from n_states with no cap (src/trex/sankoff.py
// :151-152); the state-parallel kernel (sankoff_wide.hip) stops at one 64-lane
// group per site.  Here a workgroup of 128 threads owns one tree and a tile
// of kBigT consecutive sites, which it walks one site at a time: thread i is
// parent state i, the cost matrix sits in LDS with a padded row stride (Q + 1:
// thread i reading C[i][j] and thread j reading C[i][j] are both
// bank-conflict-free), and a node's children are combined over j in a loop.
// Same semantics as every other kernel of the library:
//   * the one-wave post-order program of plan.cpp (Sethi-Ullman LDS slots,
//     register bypass -> a double-buffered "previous D" row, adjoint
//     accumulate / unreached / root flags), trex's child rules (leaf row,
//     computed internal row, 1e5 row for -1 and forward references,
//     sankoff.py:60,67,152);
//   * hard min-plus (bit-exact: C[i][j] + D[j] and min in fp32, children
//     added in trex's order) and the softmin relaxation in its per-row
//     stabilised form (exact for every cost range, no factored fast path);
//   * adjoint: the tie-averaged subgradient (tau = 0) or softmax weights,
//     dC accumulated per state row in LDS, child cotangents as column sums
//     over the parent states (thread j sums over i), marginals and first-index
//     argmax ancestral states.
// Alphabets this large are rare (trex's tests use 2-20 states), so the kernel
// is written for exactness and generality; per-tile fp64 partials feed the
// same fixed-order reduce as the other kernels.  Leaf codes and ancestral
// states stay int8 (the ABI), hence Q <= 128.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "sankoff_dev.h"
#include "trex_common.h"

namespace trex {

namespace {

constexpr int kBigT = 16;         // sites per workgroup (walked in turn)
constexpr int kBigRaggedT = 64;   // ragged batches: the plan's (tree, 64-site) items
constexpr int kBigThreads = 128;  // = the largest alphabet: thread i = state i

struct BigArgs {
  const int4* steps;  // one-wave forward program [B][n_int]
  const int8_t* leaves;
  const float* cost;
  int n_int, nl, L, tiles, B, Q, n_slots;
  float a, bcoef;
  int hard_root;
  float* dp;          // [B][n_int][L][Q]
  float* site_score;  // [B][L] or null
  const float* dts;   // [B] or null
  float* marg;        // [B][n_int][L][Q] or null
  int8_t* anc;        // [B][n_int][L] or null
  double* part_tree;  // [B * tiles] (ragged: [items])
  double* part_dc;    // [Q * Q][B * tiles] (ragged: [Q * Q][items])
  // ragged batches (trex_ragged_plan_build): per-tree records, item -> tree
  const int* rmeta;
  const int* ritem;
  int nitems;
};

// block-wide reductions over the 128 threads (two waves): min, sum, and the
// first index of the maximum
__device__ __forceinline__ float block_min(float v, float* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  float m = red[0];
  for (int k = 1; k < kBigThreads; ++k) m = fminf(m, red[k]);
  __syncthreads();
  return m;
}
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  float s = 0.0f;
  for (int k = 0; k < kBigThreads; ++k) s += red[k];
  __syncthreads();
  return s;
}
__device__ __forceinline__ int block_argmax_first(float v, bool own, float* red) {
  const int t = threadIdx.x;
  red[t] = own ? v : -INFINITY;
  __syncthreads();
  float bv = red[0];
  int bi = 0;
  for (int k = 1; k < kBigThreads; ++k)
    if (red[k] > bv) {
      bv = red[k];
      bi = k;
    }
  __syncthreads();
  return bi;
}

template <int PHASE, bool SOFT, bool RAGGED>
__global__ __launch_bounds__(kBigThreads) void sankoff_bigq_kernel(BigArgs A) {
  constexpr bool FWD = (PHASE & 1) != 0;
  constexpr bool BWD = (PHASE & 2) != 0;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int Q = A.Q, QP = Q + 1;
  const int i = threadIdx.x;  // parent state (forward) / child state (column sums)
  const bool own = i < Q;
  int ni, L, tree, tile;
  size_t leaf_base, rows_base, site_base;
  const int4* prog;
  if constexpr (RAGGED) {  // one (tree, 64-site) item of the ragged plan
    tree = A.ritem[blockIdx.x];
    const int* m = A.rmeta + (size_t)tree * kRaggedMeta;
    ni = m[1];
    L = m[3];
    site_base = (size_t)(uint32_t)m[4];
    tile = blockIdx.x - m[5];
    leaf_base = (size_t)(uint32_t)m[6] | ((size_t)(uint32_t)m[7] << 32);
    rows_base = (size_t)(uint32_t)m[8] | ((size_t)(uint32_t)m[9] << 32);
    prog = A.steps + m[0];
  } else {
    ni = A.n_int;
    L = A.L;
    tree = blockIdx.x / A.tiles;
    tile = blockIdx.x - tree * A.tiles;
    site_base = (size_t)tree * L;
    leaf_base = (size_t)tree * A.nl * L;
    rows_base = (size_t)tree * ni * L;
    prog = A.steps + (size_t)tree * ni;
  }
  constexpr int TS = RAGGED ? kBigRaggedT : kBigT;  // sites walked by this workgroup
  const int nb = RAGGED ? A.nitems : A.B * A.tiles;
  const float a = A.a, bcoef = A.bcoef;

  // ---- LDS: C [Q][Q+1] | dC [Q][Q+1] | slots [n_slots+1][Q] | prev [2][Q] |
  //      gnext [Q] | child D [Q] | mn [Q] | r [Q] | reduce [128] ----
  float* C = lds;
  float* dcl = C + Q * QP;
  float* slots = dcl + Q * QP;
  float* prev = slots + (A.n_slots + 1) * Q;
  float* gnx = prev + 2 * Q;
  float* dbuf = gnx + Q;
  float* mnb = dbuf + Q;
  float* rb = mnb + Q;
  float* red = rb + Q;
  for (int e = i; e < Q * Q; e += kBigThreads) {
    const int r = e / Q, c = e - r * Q;
    C[r * QP + c] = A.cost[e];
    dcl[r * QP + c] = 0.0f;
  }
  __syncthreads();

  const int8_t* lv = A.leaves + leaf_base;
  float* dpt = A.dp + rows_base * Q;
  const float fts = A.dts ? A.dts[tree] : 1.0f;
  double tree_part = 0.0;

  // message of one child to parent state i: min / smin_j (C[i][j] + D[j]);
  // D: dsrc (LDS row) or, for a leaf / 1e5 row, 0 at `code` and 1e5 elsewhere
  auto message = [&](const float* dsrc, int code) -> float {
    const float* ci = C + (own ? i : 0) * QP;
    float mn = INFINITY;
    for (int j = 0; j < Q; ++j) {
      const float dj = dsrc ? dsrc[j] : (j == code ? 0.0f : kSentinel);
      mn = fminf(mn, ci[j] + dj);
    }
    if (!SOFT) return mn;
    float s = 0.0f;
    for (int j = 0; j < Q; ++j) {
      const float dj = dsrc ? dsrc[j] : (j == code ? 0.0f : kSentinel);
      s += fast_exp2((mn - (ci[j] + dj)) * a);
    }
    return fmaf(-bcoef, fast_log2(s), mn);
  };
  auto leaf_code = [&](int desc, int site) -> int {
    const int c = (int)lv[(size_t)(desc & 0xFFFF) * L + site];
    return ((unsigned)c < (unsigned)Q) ? c : Q;
  };

  for (int s = 0; s < TS; ++s) {
    const int site = tile * TS + s;
    if (site >= L) break;  // uniform
    float* drow = dpt + (size_t)site * Q;  // + row * L * Q
    float dv = 0.0f;
    if constexpr (FWD) {
      for (int k = 0; k < ni; ++k) {
        const int4 stp = prog[k];
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? stp.y : stp.z;
          const int kind = (desc >> 24) & 3;
          float m;
          if (kind == kKindInt)
            m = message((desc & kChildPrev) ? prev + ((k - 1) & 1) * Q : slots + ((desc >> 16) & 0xFF) * Q, 0);
          else
            m = message(nullptr, kind == kKindLeaf ? leaf_code(desc, site) : Q);
          dv = c == 0 ? m : dv + m;
        }
        const int row = stp.x & 0xFFFF;
        if (own) drow[(size_t)row * L * Q + i] = dv;
        __syncthreads();  // every child read before a slot is reused
        const int oslot = (stp.x >> 16) & 0xFF;
        if (own) {
          prev[(k & 1) * Q + i] = dv;
          if (!(stp.w & kStepToNext) && oslot != 0xFF) slots[oslot * Q + i] = dv;
        }
        __syncthreads();
      }
    } else {
      dv = own ? drow[(size_t)(ni - 1) * L * Q + i] : 0.0f;
    }

    // ---- root: site score and cotangent (sankoff.py:187) ----
    const float mn = block_min(own ? dv : INFINITY, red);
    float groot, score;
    if (!SOFT || A.hard_root) {
      const float hit = (own && dv == mn) ? 1.0f : 0.0f;
      const float cnt = block_sum(hit, red);
      groot = hit / cnt;
      score = mn;
    } else {
      const float e = own ? fast_exp2((mn - dv) * a) : 0.0f;
      const float sm = block_sum(e, red);
      groot = e * __builtin_amdgcn_rcpf(sm);
      score = fmaf(-bcoef, fast_log2(sm), mn);
    }
    if constexpr (FWD) {
      if (i == 0) {
        if (A.site_score) A.site_score[site_base + site] = score;
        tree_part += (double)score;
      }
    }

    if constexpr (BWD) {
      if (own) slots[A.n_slots * Q + i] = groot * fts;
      __syncthreads();
      for (int k = ni - 1; k >= 0; --k) {
        const int4 stp = prog[k];
        if (stp.w & kStepUnreached) continue;  // uniform
        const int row = stp.x & 0xFFFF;
        const float g = own ? ((stp.w & kStepToNext) ? gnx[i]
                                                     : slots[((stp.w & kStepRoot) ? A.n_slots
                                                                                  : ((stp.x >> 16) & 0xFF)) * Q + i])
                            : 0.0f;
        if (A.marg && own) A.marg[(rows_base + (size_t)row * L + site) * Q + i] = g;
        if (A.anc) {
          const int bi = block_argmax_first(g, own, red);
          if (i == 0) A.anc[rows_base + (size_t)row * L + site] = (int8_t)bi;
        }
        __syncthreads();  // g read from its slot before children overwrite slots
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? stp.y : stp.z;
          const int kind = (desc >> 24) & 3;
          // the child's D row in LDS (internal rows re-read from the table)
          if (own)
            dbuf[i] = kind == kKindInt ? drow[(size_t)(desc & 0xFFFF) * L * Q + i]
                                       : (kind == kKindLeaf && i == leaf_code(desc, site) ? 0.0f : kSentinel);
          __syncthreads();
          // phase A (thread i = parent state): weights of row i, dC row i
          if (own) {
            const float* ci = C + i * QP;
            float m = INFINITY;
            for (int j = 0; j < Q; ++j) m = fminf(m, ci[j] + dbuf[j]);
            float r;
            if (!SOFT) {
              float cnt = 0.0f;
              for (int j = 0; j < Q; ++j) cnt += (ci[j] + dbuf[j] == m) ? 1.0f : 0.0f;
              r = g / cnt;
              for (int j = 0; j < Q; ++j)
                if (ci[j] + dbuf[j] == m) dcl[i * QP + j] += r;
            } else {
              float sm = 0.0f;
              for (int j = 0; j < Q; ++j) sm += fast_exp2((m - (ci[j] + dbuf[j])) * a);
              r = g * __builtin_amdgcn_rcpf(sm);
              for (int j = 0; j < Q; ++j) dcl[i * QP + j] += r * fast_exp2((m - (ci[j] + dbuf[j])) * a);
            }
            mnb[i] = m;
            rb[i] = r;
          }
          __syncthreads();
          // phase B (thread j = child state): cotangent = column sum of weights
          if (kind == kKindInt) {
            if (own) {
              const int j = i;
              const float dj = dbuf[j];
              float gc = 0.0f;
              for (int p = 0; p < Q; ++p) {
                const float x = C[p * QP + j] + dj;
                if (!SOFT)
                  gc += (x == mnb[p]) ? rb[p] : 0.0f;
                else
                  gc += rb[p] * fast_exp2((mnb[p] - x) * a);
              }
              if (desc & kChildPrev) {
                gnx[j] = gc;
              } else {
                float* sl = slots + ((desc >> 16) & 0xFF) * Q + j;
                *sl = (desc & kStepAccumulate) ? *sl + gc : gc;
              }
            }
          }
          __syncthreads();
        }
      }
    }
  }

  if constexpr (FWD) {
    if (i == 0) A.part_tree[blockIdx.x] = tree_part;
  }
  if constexpr (BWD) {
    __syncthreads();
    for (int e = i; e < Q * Q; e += kBigThreads) {
      const int r = e / Q, c = e - r * Q;
      A.part_dc[(size_t)e * nb + blockIdx.x] = (double)dcl[r * QP + c];
    }
  }
}

// trex-exact reconstruction for Q > 64 (sankoff.py:166-185, 191-267): one
// lane per site walks the host-simulated DFS order (plan.cpp), C in LDS,
// each step's DP row streamed from the table, trex's strict-< scan (the
// first argmin); parent states of visited nodes in LDS.
// Ragged batches (no bound on a tree's node count at launch) re-read the
// parent's state from this lane's own output instead of the LDS array.
template <bool RAGGED>
__global__ __launch_bounds__(kWave) void bigq_backtrack_kernel(const int* __restrict__ bt,
                                                                const float* __restrict__ cost,
                                                                const float* __restrict__ dp,
                                                                int n_int, int L, int Q, int tiles,
                                                                int8_t* __restrict__ anc,
                                                                const int* __restrict__ rmeta,
                                                                int B, int items, int steps) {
  extern __shared__ __attribute__((aligned(16))) float bl[];
  float* c = bl;                                          // [Q][Q]
  int8_t* sts = reinterpret_cast<int8_t*>(bl + Q * Q);    // [n_int][64]
  int tree, tile;
  size_t rows_base;
  if constexpr (RAGGED) {
    tree = rmeta[(size_t)B * kRaggedMeta + blockIdx.x];
    const int* m = rmeta + (size_t)tree * kRaggedMeta;
    n_int = m[1];
    L = m[3];
    tile = blockIdx.x - m[5];
    rows_base = (size_t)(uint32_t)m[8] | ((size_t)(uint32_t)m[9] << 32);
    bt = rmeta + (size_t)B * kRaggedMeta + items + (size_t)steps * 4 + (size_t)m[0] * 2;
  } else {
    tree = blockIdx.x / tiles;
    tile = blockIdx.x - tree * tiles;
    rows_base = (size_t)tree * n_int * L;
    bt += (size_t)tree * n_int * 2;
  }
  const int lane = threadIdx.x;
  for (int t = lane; t < Q * Q; t += kWave) c[t] = cost[t];
  __syncthreads();
  const int site = tile * kWave + lane;
  if (site >= L) return;
  const float* dpt = dp + rows_base * Q + (size_t)site * Q;
  int8_t* at = anc + rows_base + site;
  for (int k = 0; k < n_int; ++k) {
    const int ex = bt[2 * k], ey = bt[2 * k + 1];
    const int x = ex & 0xFFFF;
    const int kind = (ex >> 16) & 0xF;
    int out = 0;
    if (kind != kBtUnreached) {
      const float* d = dpt + (size_t)x * L * Q;
      const bool sent = kind == kBtSentinel;
      if (kind == kBtRoot) {
        float bv = d[0];
        for (int j = 1; j < Q; ++j) {
          const float v = d[j];
          if (v < bv) { bv = v; out = j; }
        }
      } else {
        const int sp = RAGGED ? (int)at[(size_t)ey * L] : (int)sts[ey * kWave + lane];
        const float* row = c + sp * Q;
        float bv = row[0] + (sent ? kSentinel : d[0]);
        for (int j = 1; j < Q; ++j) {
          const float v = row[j] + (sent ? kSentinel : d[j]);
          if (v < bv) { bv = v; out = j; }
        }
      }
    }
    if constexpr (!RAGGED) sts[x * kWave + lane] = (int8_t)out;
    at[(size_t)x * L] = (int8_t)out;
  }
}

}  // namespace

int bigq_tiles(int L) { return (L + kBigT - 1) / kBigT; }

int64_t bigq_workspace_bytes(int B, int L, int Q) {
  return (int64_t)B * bigq_tiles(L) * 8 * (1 + (int64_t)Q * Q) + 256;
}

size_t bigq_lds_bytes(int n_slots, int Q) {
  return ((size_t)2 * Q * (Q + 1) + (size_t)(n_slots + 1) * Q + 6 * (size_t)Q + kBigThreads) * 4;
}

template <bool RAGGED>
int bigq_launch(const char* fn, const BigArgs& A, const WideCall& c, int64_t nb, size_t lds) {
  hipStream_t st = (hipStream_t)c.stream;
  auto go = [&](auto kernel) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kernel, dim3((unsigned)nb), dim3(kBigThreads), lds, st, A);
  };
  if (c.soft) {
    if (c.phase == 1) go(sankoff_bigq_kernel<1, true, RAGGED>);
    else if (c.phase == 2) go(sankoff_bigq_kernel<2, true, RAGGED>);
    else go(sankoff_bigq_kernel<3, true, RAGGED>);
  } else {
    if (c.phase == 1) go(sankoff_bigq_kernel<1, false, RAGGED>);
    else if (c.phase == 2) go(sankoff_bigq_kernel<2, false, RAGGED>);
    else go(sankoff_bigq_kernel<3, false, RAGGED>);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

int bigq_run(const char* fn, const WideCall& c) {
  const int tiles = bigq_tiles(c.L);
  const size_t lds = bigq_lds_bytes(c.n_slots, c.Q);
  if (c.Q > kBigMaxQ) return set_error(TREX_E_UNSUPPORTED, "%s: Q=%d > %d", fn, c.Q, kBigMaxQ);
  if (lds > 160 * 1024) return set_error(TREX_E_UNSUPPORTED, "%s: LDS stack too deep", fn);
  if ((int64_t)c.B * tiles > 0x7FFFFFFF) return set_error(TREX_E_ARG, "%s: grid too large", fn);
  BigArgs A;
  A.steps = reinterpret_cast<const int4*>(c.steps);
  A.leaves = c.leaves;
  A.cost = c.cost;
  A.n_int = c.ni;
  A.nl = c.nl;
  A.L = c.L;
  A.tiles = tiles;
  A.B = c.B;
  A.Q = c.Q;
  A.n_slots = c.n_slots;
  A.a = c.a;
  A.bcoef = c.bcoef;
  A.hard_root = c.hard_root;
  A.dp = c.dp;
  A.site_score = c.site_score;
  A.dts = c.dts;
  A.marg = c.marg;
  A.anc = c.anc;
  const int64_t nb = (int64_t)c.B * tiles;
  A.part_tree = static_cast<double*>(c.workspace);
  A.part_dc = A.part_tree + nb;
  A.rmeta = nullptr;
  A.ritem = nullptr;
  A.nitems = 0;
  if (int e = bigq_launch<false>(fn, A, c, (int64_t)nb, lds)) return e;
  return partial_reduce(fn, A.part_tree, A.part_dc, c.B, tiles, c.Q, c.phase, c.tree_score,
                        c.d_cost, c.stream);
}

// ragged batches: the plan's (tree, 64-site) items, per-item partials summed
// per tree by the ragged partial reduce
int bigq_ragged_run(const char* fn, const WideCall& c, const int* rmeta, const int* ritem,
                    int64_t items) {
  const size_t lds = bigq_lds_bytes(c.n_slots, c.Q);
  if (c.Q > kBigMaxQ) return set_error(TREX_E_UNSUPPORTED, "%s: Q=%d > %d", fn, c.Q, kBigMaxQ);
  if (lds > 160 * 1024) return set_error(TREX_E_UNSUPPORTED, "%s: LDS stack too deep", fn);
  BigArgs A;
  A.steps = reinterpret_cast<const int4*>(c.steps);
  A.leaves = c.leaves;
  A.cost = c.cost;
  A.n_int = 0;
  A.nl = c.nl;
  A.L = 0;
  A.tiles = 0;
  A.B = c.B;
  A.Q = c.Q;
  A.n_slots = c.n_slots;
  A.a = c.a;
  A.bcoef = c.bcoef;
  A.hard_root = c.hard_root;
  A.dp = c.dp;
  A.site_score = c.site_score;
  A.dts = c.dts;
  A.marg = c.marg;
  A.anc = c.anc;
  A.part_tree = static_cast<double*>(c.workspace);
  A.part_dc = A.part_tree + items;
  A.rmeta = rmeta;
  A.ritem = ritem;
  A.nitems = (int)items;
  if (int e = bigq_launch<true>(fn, A, c, items, lds)) return e;
  return partial_reduce(fn, A.part_tree, A.part_dc, c.B, 0, c.Q, c.phase, c.tree_score, c.d_cost,
                        c.stream, rmeta + 5, kRaggedMeta, (int)items);
}

int bigq_backtrack(const int32_t* bt, const float* cost, const float* dp, int B, int L, int ni,
                   int Q, int8_t* anc, void* stream) {
  const int tiles = (L + kWave - 1) / kWave;
  const size_t lds = (size_t)Q * Q * 4 + (size_t)ni * kWave;
  if (lds > 160 * 1024)
    return set_error(TREX_E_UNSUPPORTED, "trex_sankoff_backtrack: %d internal nodes at Q=%d", ni, Q);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(bigq_backtrack_kernel<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(bigq_backtrack_kernel<false>, dim3((unsigned)((int64_t)B * tiles)), dim3(kWave),
                     lds, (hipStream_t)stream, bt, cost, dp, ni, L, Q, tiles, anc, nullptr, 0, 0, 0);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "trex_sankoff_backtrack: %s", hipGetErrorString(e));
  return TREX_OK;
}

int bigq_ragged_backtrack(const int32_t* rmeta, int B, int64_t items, int64_t steps,
                          const float* cost, const float* dp, int Q, int8_t* anc, void* stream) {
  const size_t lds = (size_t)Q * Q * 4;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(bigq_backtrack_kernel<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(bigq_backtrack_kernel<true>, dim3((unsigned)items), dim3(kWave), lds,
                     (hipStream_t)stream, nullptr, cost, dp, 0, 0, Q, 0, anc, rmeta, B, (int)items,
                     (int)steps);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_error(TREX_E_HIP, "trex_sankoff_ragged_backtrack: %s", hipGetErrorString(e));
  return TREX_OK;
}

}  // namespace trex
