// libtrexhip.so -- staged Sankoff kernel for small grids (gfx950).
//
// Same semantics as sankoff.hip / sankoff_wide.hip (trex src/trex/sankoff.py
// run_dp :24-94, run_sankoff :114-188, build-defined softmin adjoint), for
// launches with too few work items to fill the chip: C2 is ONE 64-taxon tree
// x 10 000 sites, 625 16-site items for 1 024 SIMDs, and each item's wave
// walks all 63 internal nodes serially forward and again in reverse.
//
// Here one work item (one tree x one site group of 64 / G sites, G lanes per
// site as in sankoff_wide.hip) is a workgroup of kStageWaves waves.  The
// planner levels the tree by height (plan.cpp stage_one_tree): a stage's
// nodes depend only on earlier stages, so the waves evaluate them in
// parallel and meet at an LDS barrier; the serial chain is the tree height
// (balanced 64 taxa: 6 stages, at most 4 nodes per wave in the widest)
// instead of 63 nodes, in both sweeps.
//   * every internal row's D vector stays in LDS ([n_int][64] floats; the
//     DP table is still written to HBM as trex returns it), so the adjoint
//     reads no DP row from HBM; cotangents have their own [n_int][64] slots
//     (a shared child of trex's DAG quirk accumulates from several parents:
//     such trees are scheduled serially on wave 0, plan.cpp);
//   * stage barriers wait on LDS traffic only (s_waitcnt lgkmcnt(0);
//     s_barrier): the DP-table stores stay in flight across stages;
//   * dC: each wave sums its groups, the workgroup sums its waves in a fixed
//     order in LDS and writes one partial per item, reduced by the same
//     fixed-order kernel as the other paths (bitwise reproducible).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "sankoff_dev.h"
#include "trex_common.h"
#include "wide_dev.h"

namespace trex {

namespace {

constexpr int kSW = kStageWaves;

struct SArgs {
  const int* staged;  // per-tree staged regions (trex_common.h)
  int64_t stride;     // ints per region
  const int8_t* leaves;
  const float* cost;
  int n_int, nl, L, tiles, B, Q;
  float a, bcoef;
  int hard_root;
  float* dp;          // [B][n_int][L][Q]
  float* site_score;  // [B][L] or null
  const float* dts;   // [B] or null
  float* marg;        // [B][n_int][L][Q] or null
  int8_t* anc;        // [B][n_int][L] or null
  double* part_tree;  // [B * tiles]
  double* part_dc;    // [Q * Q][B * tiles]
  unsigned* counter;  // arrival counter (workspace, zero between launches)
  int tail;           // 1: the last workgroup reduces the partials
  float* tree_score;  // [B]
  float* d_cost;      // [Q][Q]
  const int* skip = nullptr;  // matrix-core kernel's flag: set -> it handled this launch
};

#ifdef TREX_STAGED_TIMING
// diagnostic build (tools/build_ab.sh stagetime sankoff_staged.hip -DTREX_STAGED_TIMING): wave 0 of each of the first 4096
// workgroups stamps s_memtime at phase boundaries
__device__ unsigned long long g_stage_t[4096][20];
__device__ unsigned long long g_stage_rt[4096][2];  // s_memrealtime (100 MHz) at start / end
#define STAGE_RT(j)                                                              \
  do {                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 4096)                                 \
      g_stage_rt[blockIdx.x][j] = __builtin_amdgcn_s_memrealtime();            \
  } while (0)
#define STAGE_STAMP(j)                                                         \
  do {                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 4096 && (j) < 20)                     \
      g_stage_t[blockIdx.x][j] = __builtin_amdgcn_s_memtime();                 \
  } while (0)
#else
#define STAGE_STAMP(j) \
  do {                 \
  } while (0)
#define STAGE_RT(j) \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int G>
__host__ __device__ constexpr int staged_xchg_floats() {
  return G == 4 ? 0 : kSW * kXchg;  // G = 4 exchanges through DPP quads
}

template <int G, int MODE, int PHASE, bool LFAST>
__device__ __forceinline__ void staged_body(const SArgs& A, const WCoef<G>& cf_in, float* lds) {
  constexpr bool SOFT = MODE != kHard;
  constexpr bool FWD = (PHASE & 1) != 0;
  constexpr bool BWD = (PHASE & 2) != 0;
  constexpr int SPW = kWave / G;
  const int Q = A.Q;
  const int ni = A.n_int;
  const int tree = blockIdx.x / A.tiles;
  const int tile = blockIdx.x - tree * A.tiles;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x % kWave;
  const int grp = lane / G;
  WLane w;
  w.lane = lane;
  w.i = lane - grp * G;
  w.gbase = (grp < SPW ? grp : 0) * G;
  w.pad = w.i >= Q;
  const int site = tile * SPW + grp;
  const bool active = grp < SPW && site < A.L;
  const int L = A.L;
  const float a = A.a, bcoef = A.bcoef;

  float* X = lds + (G == 4 ? 0 : wv * kXchg);
  float* tab = lds + staged_xchg_floats<G>();  // T[code][i]
  float* ctab = tab + wide_col_table_offset(G, Q);  // G > 4: lane columns of C / K
  WCoef<G> cf = cf_in;
  cf.cl = ctab + (w.i < G ? w.i : 0) * G;
  float* itab = tab + (Q + 1) * G;             // IK[code][i]
  float* dsl = tab + wide_tab_floats(G, Q);    // D of internal row r: dsl[r * 64 + lane]
  float* gsl = dsl + (size_t)ni * kWave;       // cotangents (BWD)
  int8_t* lleaf = reinterpret_cast<int8_t*>(gsl + (BWD ? (size_t)ni * kWave : 0));

  const cptr<int> prog = as_const(A.staged) + (size_t)tree * A.stride;
  const int S = prog[4 * ni];
  const cptr<int> offs = prog + 4 * ni + 1;
  // this wave's [lo, hi) step range of stage s sits in lane s of two VGPRs
  // (one vector load up front; v_readlane per stage, no load on the chain)
  int vlo = 0, vhi = 0;
  {
    const int* og = A.staged + (size_t)tree * A.stride + 4 * ni + 1;
    if (lane < S) {
      vlo = og[lane * kSW + wv];
      vhi = og[lane * kSW + wv + 1];
    }
  }
  auto stage_range = [&](int s, int& lo, int& hi) {
    if (s < kWave) {
      lo = __builtin_amdgcn_readlane(vlo, s);
      hi = __builtin_amdgcn_readlane(vhi, s);
    } else {
      lo = offs[s * kSW + wv];
      hi = offs[s * kSW + wv + 1];
    }
  };
  // ... and, when they fit (<= 64 stages and steps), this wave's step words
  // themselves: lane t holds the wave's t-th step (stages in order), read
  // with v_readlane -- no scalar load (and lgkmcnt wait) on the chain
  int vbase = 0, sx = 0, sy = 0, sz = 0, sw = 0;
  bool regsteps;
  {
    const int cnt = vhi - vlo;  // 0 in lanes >= S
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int t = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += t;
    }
    vbase = incl - cnt;
    const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
    regsteps = S <= kWave && total <= kWave;
    if (regsteps) {
      int k = -1;
      for (int s2 = 0; s2 < S; ++s2) {
        const int b = __builtin_amdgcn_readlane(vbase, s2);
        const int lo = __builtin_amdgcn_readlane(vlo, s2);
        const int c = __builtin_amdgcn_readlane(vhi, s2) - lo;
        if (lane >= b && lane < b + c) k = lo + lane - b;
      }
      if (k >= 0) {
        // (regions are 4-byte aligned only: four dword loads)
        const int* e = A.staged + (size_t)tree * A.stride + 4 * k;
        sx = e[0];
        sy = e[1];
        sz = e[2];
        sw = e[3];
      }
    }
  }
  auto reg_step = [&](int t) {
    return I4{__builtin_amdgcn_readlane(sx, t), __builtin_amdgcn_readlane(sy, t),
              __builtin_amdgcn_readlane(sz, t), __builtin_amdgcn_readlane(sw, t)};
  };
  const uint32_t rowbytes = (uint32_t)L * Q * 4;
  const uint32_t treebytes = (uint32_t)ni * rowbytes;
  const rsrc_t rdp = make_rsrc(A.dp + (size_t)tree * ni * L * Q, treebytes);
  // inactive sites and padded states address past the buffer: stores drop, loads give 0
  const int voff = (active && !w.pad) ? (site * Q + w.i) * 4 : 0x7FFFFFF0;
  const int lgrp = grp < SPW ? grp : 0;
  STAGE_STAMP(0);
  STAGE_RT(0);

  // G = 4 with exact leaf weights: every wave keeps the leaf coefficients of
  // its lane in registers instead of reading the LDS tables on the chain:
  // crow[j] = C[i][j] (leaf message), sentm = message of the all-1e5 row,
  // ikx[j] / wm[j] = adjoint factor of a present / missing leaf state for
  // accumulator slot j (wm: the all-1e5 row's weights per unit cotangent)
  constexpr bool REGLEAF = G == 4 && LFAST;
  float crow[G], ikx[G], wm[G], sentm = 0.0f;
  if constexpr (REGLEAF) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int col = acc_col<G, MODE>(w.i, j);
      crow[j] = (w.pad || j >= Q) ? INFINITY : A.cost[w.i * Q + j];
      const float cc = (w.pad || col >= Q) ? 0.0f : A.cost[w.i * Q + col];
      ikx[j] = (w.pad || col >= Q) ? 0.0f : (MODE == kSoftK ? fast_exp2((cc - cf.cmin) * a) : 1.0f);
      wm[j] = 0.0f;
    }
    sentm = wmsg<G, MODE>(cf, X, w, a, bcoef, kSentinel);
    if constexpr (BWD) (void)wadj<G, MODE>(cf, X, w, a, kSentinel, 1.0f, wm);
  }

  // ---- prologue: leaf tables (wave 0), leaf tile, (adjoint only) D rows ----
  if (!REGLEAF && wv == 0) {
    const float sent = wmsg<G, MODE>(cf, X, w, a, bcoef, kSentinel);
    if (grp == 0) {
      for (int code = 0; code < Q; ++code) {
        const float cv = w.pad ? INFINITY : A.cost[w.i * Q + code];
        tab[code * G + w.i] = cv;
        if constexpr (MODE == kSoftK) itab[code * G + w.i] = w.pad ? 0.0f : fast_exp2((cv - cf.cmin) * a);
      }
      tab[Q * G + w.i] = sent;
      fill_col_table<G, MODE>(ctab, A.cost, Q, w.i, cf.cmin, a);
    }
  }
  {
    const int8_t* lv = A.leaves + (size_t)tree * A.nl * L;
    for (int t = threadIdx.x; t < A.nl * SPW; t += kSW * kWave) {
      const int leaf = t / SPW;
      const int s = tile * SPW + (t - leaf * SPW);
      int code = s < L ? (int)lv[(size_t)leaf * L + s] : Q;
      code = ((unsigned)code < (unsigned)Q) ? code : Q;
      lleaf[t] = (int8_t)code;
    }
  }
  if constexpr (!FWD) {
    for (int r = wv; r < ni; r += kSW)
      dsl[r * kWave + lane] =
          __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rdp, voff, r * rowbytes, 0));
  }
  __syncthreads();
  STAGE_STAMP(1);

  // ---- forward: stage by stage, each wave its own node list ----
  if constexpr (FWD) {
    for (int s = 0; s < S; ++s) {
      int lo, hi;
      stage_range(s, lo, hi);
      const int sb = __builtin_amdgcn_readlane(vbase, s < kWave ? s : 0) - lo;
      I4 nxt = regsteps ? I4{0, 0, 0, 0} : load_step(prog, lo < hi ? lo : 0);
      for (int k = lo; k < hi; ++k) {
        I4 stp;
        if (regsteps) {
          stp = reg_step(sb + k);
        } else {
          stp = nxt;
          if (k + 1 < hi) nxt = load_step(prog, k + 1);
        }
        float dv = 0.0f;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? stp.y : stp.z;
          const int kind = (desc >> 24) & 3;
          float m;
          if (kind == kKindLeaf) {
            const int code = lleaf[(desc & 0xFFFF) * SPW + lgrp];
            if constexpr (REGLEAF) {
              m = sentm;
#pragma unroll
              for (int j = 0; j < G; ++j) m = (code == j && j < Q) ? crow[j] : m;  // code Q: missing
            } else if constexpr (LFAST) {
              m = tab[code * G + w.i];
            } else {
              m = wmsg<G, MODE>(cf, X, w, a, bcoef, code == w.i ? 0.0f : kSentinel);
            }
          } else if (kind == kKindInt) {
            m = wmsg<G, MODE>(cf, X, w, a, bcoef, dsl[(desc & 0xFFFF) * kWave + lane]);
          } else {
            if constexpr (REGLEAF)
              m = sentm;
            else
              m = tab[Q * G + w.i];
          }
          dv = (c == 0) ? m : dv + m;
        }
        const int row = stp.x & 0xFFFF;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dv), rdp, voff, row * rowbytes, 0);
        dsl[row * kWave + lane] = dv;
      }
      lds_barrier();
      STAGE_STAMP(2 + s);
    }
  }

  // ---- root (last internal row): score + cotangent (sankoff.py:187), wave 0 ----
  if (wv == 0) {
    const float dv = dsl[(ni - 1) * kWave + lane];
    float groot, score;
    float d[G];
    xchg<G>(X, lane, w.gbase, w.pad ? INFINITY : dv, d);
    float mn = d[0];
#pragma unroll
    for (int j = 1; j < G; ++j) mn = fminf(mn, d[j]);
    if (!SOFT || A.hard_root) {
      float cnt = 0.0f;
#pragma unroll
      for (int j = 0; j < G; ++j) cnt += (d[j] == mn) ? 1.0f : 0.0f;
      groot = (!w.pad && dv == mn) ? 1.0f / cnt : 0.0f;
      score = mn;
    } else {
      const float e = w.pad ? 0.0f : fast_exp2((mn - dv) * a);
      float ee[G];
      xchg<G>(X + kWave, lane, w.gbase, e, ee);
      float s = 0.0f;
#pragma unroll
      for (int j = 0; j < G; ++j) s += ee[j];
      groot = e * __builtin_amdgcn_rcpf(s);
      score = fmaf(-bcoef, fast_log2(s), mn);
    }
    const bool leader = active && w.i == 0;
    if constexpr (FWD) {
      if (leader && A.site_score) A.site_score[(size_t)tree * L + site] = score;
      const double tot = wave_sum(leader ? (double)score : 0.0);
      if (lane == 0) store_sc1(A.part_tree + blockIdx.x, tot);
    }
    if constexpr (BWD) {
      const float dscale = A.dts ? as_const(A.dts)[tree] : 1.0f;
      gsl[(ni - 1) * kWave + lane] = active ? groot * dscale : 0.0f;
    }
  }

  if constexpr (BWD) {
    lds_barrier();
    STAGE_STAMP(10);
    float acc[G];
#pragma unroll
    for (int j = 0; j < G; ++j) acc[j] = 0.0f;
    const bool want_marg = A.marg != nullptr;
    const rsrc_t rmg = make_rsrc(want_marg ? A.marg + (size_t)tree * ni * L * Q : A.dp, treebytes);
    const bool want_anc = A.anc != nullptr;
    int8_t* at = want_anc ? A.anc + (size_t)tree * ni * L + site : nullptr;
    const bool leader = active && w.i == 0;
    for (int s = S - 1; s >= 0; --s) {
      int lo, hi;
      stage_range(s, lo, hi);
      const int sb = __builtin_amdgcn_readlane(vbase, s < kWave ? s : 0) - lo;
      I4 nxt = regsteps ? I4{0, 0, 0, 0} : load_step(prog, lo < hi ? hi - 1 : 0);
      for (int k = hi - 1; k >= lo; --k) {
        I4 stp;
        if (regsteps) {
          stp = reg_step(sb + k);
        } else {
          stp = nxt;
          if (k > lo) nxt = load_step(prog, k - 1);
        }
        if (stp.w & kStepUnreached) continue;
        const int row = stp.x & 0xFFFF;
        const float g = gsl[row * kWave + lane];
        if (want_marg)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g), rmg, voff, row * rowbytes, 0);
        if (want_anc) {
          const int bi = group_argmax<G>(X, w, w.pad ? -INFINITY : g);
          if (leader) at[(size_t)row * L] = (int8_t)bi;
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? stp.y : stp.z;
          const int kind = (desc >> 24) & 3;
          if (kind == kKindLeaf) {
            const int code = lleaf[(desc & 0xFFFF) * SPW + lgrp];
            bool onehot = false;
            if constexpr (REGLEAF) {
              // present state: dC[i][code] += g_i (/ K[i][code]); missing
              // (all-1e5 row): g_i times that row's weights
              const float gm = code == Q ? g : 0.0f;
#pragma unroll
              for (int j = 0; j < G; ++j) {
                const bool hit = code != Q && acc_col<G, MODE>(w.i, j) == code;
                acc[j] = fmaf(hit ? g : gm, hit ? ikx[j] : wm[j], acc[j]);
              }
              continue;
            }
            if constexpr (LFAST) onehot = !__any(active && code == Q);
            if (onehot) {
              // exact leaf weights are one-hot: dC[i][code] += g_i (/ K[i][code])
              float t = g;
              // (code Q only at sites past L, whose cotangent is 0: IK has no row Q)
            if constexpr (MODE == kSoftK) t = code < Q ? g * itab[code * G + w.i] : 0.0f;
              if (w.pad) t = 0.0f;
              onehot_add<G, MODE>(acc, w.i, code, t);
            } else {
              (void)wadj<G, MODE>(cf, X, w, a, code == w.i ? 0.0f : kSentinel, g, acc);
            }
          } else if (kind == kKindInt) {
            const int cs = (desc & 0xFFFF) * kWave + lane;
            float gc = wadj<G, MODE>(cf, X, w, a, dsl[cs], g, acc);
            if (desc & kStepAccumulate) gc += gsl[cs];
            gsl[cs] = gc;
          } else {
            if constexpr (REGLEAF) {
#pragma unroll
              for (int j = 0; j < G; ++j) acc[j] = fmaf(g, wm[j], acc[j]);
            } else {
              (void)wadj<G, MODE>(cf, X, w, a, kSentinel, g, acc);
            }
          }
        }
      }
      lds_barrier();
      STAGE_STAMP(11 + (S - 1 - s));
    }

    // ---- dC partial of the item: groups of a wave, then waves, in order ----
    double* red = reinterpret_cast<double*>(dsl);  // D slots are dead now
    const int Q2 = Q * Q;
#pragma unroll
    for (int j = 0; j < G; ++j) {
      double t;
      if constexpr ((SPW & (SPW - 1)) == 0) {
        // power-of-two group count: xor butterfly over the groups (lanes
        // l ^ G*2^k hold the same state i), fixed association
        float v = acc[j];
#pragma unroll
        for (int off = G; off < kWave; off <<= 1) v += __shfl_xor(v, off, kWave);
        t = (double)v;
      } else {
        const double v = (double)acc[j];
        t = v;
#pragma unroll
        for (int gq = 1; gq < SPW; ++gq) t += __shfl(v, w.i + gq * G, kWave);
      }
      if constexpr (MODE == kSoftK) t *= (double)cf.row[j];
      const int col = acc_col<G, MODE>(w.i, j);
      if (grp == 0 && !w.pad && col < Q) red[wv * Q2 + w.i * Q + col] = t;
    }
    lds_barrier();
    const int nb = A.B * A.tiles;
    for (int q = threadIdx.x; q < Q2; q += kSW * kWave) {
      double t = red[q];
#pragma unroll
      for (int v = 1; v < kSW; ++v) t += red[v * Q2 + q];
      store_sc1(A.part_dc + (size_t)q * nb + blockIdx.x, t);
    }
    STAGE_STAMP(19);
  }
  STAGE_RT(1);

  // ---- last workgroup: fixed-order sums of every item's partials.
  // Partials are written and read at device scope (sc1) and each wave waits
  // for its own stores before the arrival count: no agent-scope fence (an
  // L2 write-back per workgroup).  The counter lives in the zero-initialised
  // workspace and is reset for the next launch (graph replays).  Large
  // reductions (A.tail == 0) are left to partial_reduce's kernel. ----
  if (!A.tail) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(tab);  // leaf tables are dead now
  if (threadIdx.x == 0)
    flag[0] = __hip_atomic_fetch_add(A.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
              gridDim.x - 1;
  __syncthreads();
  if (flag[0]) {
    // entries: tree scores [0, ntree) (tiles items each), dC [ntree, nent)
    // (B * tiles items each); tpe threads per entry, each summing a fixed
    // stride of items with four accumulators (all loads independent), then
    // the entry's first thread adds the tpe partials in order
    constexpr int T = kSW * kWave;
    double* red2 = reinterpret_cast<double*>(dsl);  // [T]
    const int ntree = FWD ? A.B : 0;
    const int nent = ntree + (BWD ? Q * Q : 0);
    const int nb = A.B * A.tiles;
    const int tpe = nent >= T ? 1 : T / nent;
    const int epr = T / tpe;
    const int j = threadIdx.x % tpe;
    for (int e0 = 0; e0 < nent; e0 += epr) {
      const int e = e0 + threadIdx.x / tpe;
      const bool live = threadIdx.x / tpe < epr && e < nent;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      if (live) {
        const double* src = e < ntree ? A.part_tree + (size_t)e * A.tiles
                                      : A.part_dc + (size_t)(e - ntree) * nb;
        const int n = e < ntree ? A.tiles : nb;
        int k = j;
        for (; k + 3 * tpe < n; k += 4 * tpe) {
          a0 += load_sc1(src + k);
          a1 += load_sc1(src + k + tpe);
          a2 += load_sc1(src + k + 2 * tpe);
          a3 += load_sc1(src + k + 3 * tpe);
        }
        for (; k < n; k += tpe) a0 += load_sc1(src + k);
      }
      red2[threadIdx.x] = (a0 + a1) + (a2 + a3);
      __syncthreads();
      if (live && j == 0) {
        double v = red2[threadIdx.x];
        for (int q = 1; q < tpe; ++q) v += red2[threadIdx.x + q];
        if (e < ntree)
          A.tree_score[e] = (float)v;
        else
          A.d_cost[e - ntree] = (float)v;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) __hip_atomic_store(A.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int G, int MODE, int PHASE>
__device__ __forceinline__ void staged_dispatch_leaf(const SArgs& A, const WCoef<G>& cf, float cmax,
                                                     float* lds) {
  const float range = cmax - cf.cmin;
  const bool lfast = (MODE != kHard) ? ((kSentinel - range) * A.a >= 64.0f) : (range < 99000.0f);
  if (lfast)
    staged_body<G, MODE, PHASE, true>(A, cf, lds);
  else
    staged_body<G, MODE, PHASE, false>(A, cf, lds);
}

// G = 4 (C2): at most 80 VGPRs, so three 8-wave workgroups share a CU
// (6 waves / SIMD) and C2's 625 items run in one round on 256 CUs
template <int G>
constexpr int staged_min_waves() { return G == 4 ? 6 : 1; }

template <int G, bool SOFT, int PHASE>
__global__ __launch_bounds__(kSW* kWave, staged_min_waves<G>()) void sankoff_staged_kernel(SArgs A) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (A.skip && __hip_atomic_load(A.skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int Q = A.Q;
  const int i = (threadIdx.x % kWave) % G;
  float cmin, cmax;
  cost_range<G>(A.cost, Q, i, cmin, cmax);
  if constexpr (!SOFT) {
    staged_dispatch_leaf<G, kHard, PHASE>(A, make_coefs<G, kHard>(A.cost, Q, i, cmin, A.a), cmax, lds);
  } else if (use_ktrick(cmin, cmax, A.a)) {
    staged_dispatch_leaf<G, kSoftK, PHASE>(A, make_coefs<G, kSoftK>(A.cost, Q, i, cmin, A.a), cmax, lds);
  } else {
    staged_dispatch_leaf<G, kSoftDirect, PHASE>(A, make_coefs<G, kSoftDirect>(A.cost, Q, i, cmin, A.a), cmax,
                                    lds);
  }
}

template <int G, bool SOFT>
void launch_staged(int phase, int grid, size_t lds, hipStream_t st, const SArgs& A) {
  auto go = [&](auto kernel) {
    if (lds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kSW * kWave), lds, st, A);
  };
  if (phase == 1)
    go(sankoff_staged_kernel<G, SOFT, 1>);
  else if (phase == 2)
    go(sankoff_staged_kernel<G, SOFT, 2>);
  else
    go(sankoff_staged_kernel<G, SOFT, 3>);
}

template <int G>
void launch_staged_g(int phase, bool soft, int grid, size_t lds, hipStream_t st, const SArgs& A) {
  if (soft)
    launch_staged<G, true>(phase, grid, lds, st, A);
  else
    launch_staged<G, false>(phase, grid, lds, st, A);
}

template <int G>
size_t staged_lds_g(int ni, int nl, int Q, int phase) {
  const size_t slots = (size_t)ni * kWave * ((phase & 2) ? 2 : 1);
  // dC partials [W][Q*Q] and the last workgroup's [512] sums: doubles
  // aliasing the slots
  const size_t red = std::max<size_t>((phase & 2) ? (size_t)kSW * Q * Q * 2 : 0, 2 * 256 * 2);
  const size_t b = (size_t)(staged_xchg_floats<G>() + wide_tab_floats(G, Q) + std::max(slots, red)) * 4 +
                   (size_t)nl * (kWave / G);
  return (b + 15) & ~(size_t)15;
}

}  // namespace

#ifdef TREX_STAGED_TIMING
extern "C" int trex_debug_stage_times(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stage_t), sizeof(g_stage_t)) == hipSuccess ? 0 : -4;
}
extern "C" int trex_debug_stage_rt(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stage_rt), sizeof(g_stage_rt)) == hipSuccess ? 0 : -4;
}
#endif

size_t staged_lds_bytes(int ni, int nl, int Q, int phase) {
  if (Q > 32) return ~(size_t)0;  // codons: one site per wave already, wide kernel
  switch (wide_group(Q)) {
    case 4: return staged_lds_g<4>(ni, nl, Q, phase);
    case 8: return staged_lds_g<8>(ni, nl, Q, phase);
    case 16: return staged_lds_g<16>(ni, nl, Q, phase);
    case 20: return staged_lds_g<20>(ni, nl, Q, phase);
    default: return staged_lds_g<32>(ni, nl, Q, phase);
  }
}

int staged_run(const char* fn, const WideCall& c, const int32_t* staged) {
  if (c.Q > 32) return set_error(TREX_E_UNSUPPORTED, "%s: staged kernel needs Q <= 32", fn);
  const int tiles = wide_tiles(c.L, c.Q);
  const size_t lds = staged_lds_bytes(c.ni, c.nl, c.Q, c.phase);
  if (lds > 160 * 1024) return set_error(TREX_E_UNSUPPORTED, "%s: staged LDS too large", fn);
  if ((int64_t)c.B * tiles > 0x7FFFFFFF) return set_error(TREX_E_ARG, "%s: grid too large", fn);
  if ((int64_t)c.ni * c.L * c.Q * 4 > 0x7FFFFFF0LL)
    return set_error(TREX_E_UNSUPPORTED, "%s: one tree's DP table exceeds 2 GiB", fn);
  SArgs A;
  A.staged = staged;
  A.stride = staged_tree_ints(c.ni);
  A.leaves = c.leaves;
  A.cost = c.cost;
  A.n_int = c.ni;
  A.nl = c.nl;
  A.L = c.L;
  A.tiles = tiles;
  A.B = c.B;
  A.Q = c.Q;
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
  // the counter sits in the workspace's tail slack (wide_workspace_bytes)
  A.counter = reinterpret_cast<unsigned*>(A.part_dc + nb * c.Q * c.Q);
  A.tree_score = c.tree_score;
  A.d_cost = c.d_cost;
  // in-kernel tail for small reductions (C2: 17 entries x 625 items);
  // larger ones go to the separate fixed-order reduce kernel
  const int64_t nent = ((c.phase & 1) ? c.B : 0) + ((c.phase & 2) ? (int64_t)c.Q * c.Q : 0);
  // (behind the matrix-core kernel the separate reduce runs: it knows, from
  // the device flag, whose partials to sum)
  A.tail = !c.mx_flag && nent * nb <= (int64_t)1 << 16;
  A.skip = c.mx_flag;
  hipStream_t st = (hipStream_t)c.stream;
  const int grid = (int)nb;
  switch (wide_group(c.Q)) {
    case 4: launch_staged_g<4>(c.phase, c.soft, grid, lds, st, A); break;
    case 8: launch_staged_g<8>(c.phase, c.soft, grid, lds, st, A); break;
    case 16: launch_staged_g<16>(c.phase, c.soft, grid, lds, st, A); break;
    case 20: launch_staged_g<20>(c.phase, c.soft, grid, lds, st, A); break;
    default: launch_staged_g<32>(c.phase, c.soft, grid, lds, st, A); break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  if (A.tail) return TREX_OK;  // partials reduced by the kernel's last workgroup
  return partial_reduce(fn, A.part_tree, A.part_dc, c.B, tiles, c.Q, c.phase, c.tree_score,
                        c.d_cost, c.stream, nullptr, 0, 0, 1, c.mx_flag, c.mx_tiles);
}

}  // namespace trex
