// libtrexhip.so -- Sankoff DP for Q > 4 states (protein: Q = 20), gfx950.
//
// Same semantics as sankoff.hip (trex src/trex/sankoff.py run_dp :24-94,
// run_sankoff :114-188, backtrack :191-267, and the build-defined softmin
// adjoint), different mapping.  With Q = 20 a lane-per-site kernel would hold
// Q^2 = 400 dC accumulators per lane; here the STATE axis is spread over
// lanes instead:
//   * a group of G lanes (G = 8 / 16 / 20 / 32 >= Q) owns one site, lane i of
//     the group owns parent state i; a 64-lane wave holds 64 / G sites;
//   * lane i keeps row i and column i of C (or of K = exp(-(C - cmin)/tau))
//     in VGPRs and accumulates row i of dC -- G accumulators per lane;
//   * the all-to-all inside a site (every parent state needs every child
//     state) goes through a 64-float LDS exchange buffer per wave: one
//     ds_write_b32 + G/4 ds_read_b128 per exchanged vector;
//   * the DP table is site-major, [B][n_int][L][Q]: a wave's row store is
//     64/G * Q * 4 contiguous bytes.
// Padded states (Q < G) are inert: their D is +inf on every exchange, their
// cotangent 0, their C entries +inf / K entries 0.
// Partial sums go to the workspace per wave and are reduced by a second,
// fixed-order kernel (bitwise reproducible, no counters).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "sankoff_dev.h"
#include "trex_common.h"
#include "wide_dev.h"

namespace trex {

namespace {

struct WArgs {
  const int* steps;  // [B][n_int] x int4 (plan.cpp)
  const int8_t* leaves;
  const float* cost;
  int n_int, nl, L, tiles, B, n_slots, Q;
  float a, bcoef;
  int hard_root;
  float* dp;          // [B][n_int][L][Q]
  float* site_score;  // [B][L] or null
  const float* dts;   // [B] or null
  float* marg;        // [B][n_int][L][Q] or null
  int8_t* anc;        // [B][n_int][L] or null
  double* part_tree;  // [B * tiles] (ragged: [items * wpi])
  double* part_dc;    // [Q * Q][grid]
  // ragged batches (plan.cpp trex_ragged_plan_build): per-tree records and
  // the 64-site work item -> tree table; wpi waves per item (SPW sites each)
  const int* rmeta;
  const int* ritem;
  int wpi;
  const int* skip = nullptr;  // matrix-core kernel's flag: set -> it handled this launch
  // gate of the lane-per-site kernel launched behind this one (site_gate_write):
  // non-null -> decide per workgroup, workgroup 0 writes K / K^T / flag
  int* site_flag = nullptr;
  float* site_kg = nullptr;
  int nitems = 0;  // work items = the grid (partials are [item] / [Q*Q][item])
};

// LDS map (floats): 4 exchange buffers [4][64], leaf message table
// T[Q + 1][G] (row Q = message of the all-1e5 row), IK[Q][G] = 1 / K[i][code],
// slots [n_slots + 1][64] (n_slots = root cotangent), leaf tile [nl][64/G] i8
// (exchange helpers, wmsg / wadj: wide_dev.h)

template <int G, int MODE, int PHASE, bool LFAST, bool SYM, bool RAGGED>
__device__ __forceinline__ void wide_body(const WArgs& A, const WCoef<G>& cf_in, float* lds,
                                          const int blk) {
  constexpr bool SOFT = MODE != kHard;
  constexpr bool FWD = (PHASE & 1) != 0;
  constexpr bool BWD = (PHASE & 2) != 0;
  constexpr int SPW = kWave / G;
  const int Q = A.Q;
  const int lane = threadIdx.x;
  const int grp = lane / G;
  WLane w;
  w.lane = lane;
  w.i = lane - grp * G;
  w.gbase = (grp < SPW ? grp : 0) * G;
  w.pad = w.i >= Q;
  // this wave's tree, shape and site groups: uniform batches tile each tree
  // in SPW-site items; ragged batches split each 64-site item of the plan
  // into wpi waves of SPW sites
  int tree, n_int, nl, L, site0;
  size_t leaf_base, rows_base, site_base;
  const int* steps;
  int in_item = SPW;  // groups of this wave inside the item
  if constexpr (RAGGED) {
    const int item = blk / A.wpi;
    const int sub = blk - item * A.wpi;
    tree = as_const(A.ritem)[item];
    const cptr<int> m = as_const(A.rmeta) + (size_t)tree * kRaggedMeta;
    n_int = m[1];
    nl = m[2];
    L = m[3];
    site_base = (size_t)(uint32_t)m[4];
    site0 = (item - m[5]) * kWave + sub * SPW;
    in_item = kWave - sub * SPW;
    leaf_base = (size_t)(uint32_t)m[6] | ((size_t)(uint32_t)m[7] << 32);
    rows_base = (size_t)(uint32_t)m[8] | ((size_t)(uint32_t)m[9] << 32);
    steps = A.steps + (size_t)m[0] * 4;
  } else {
    tree = blk / A.tiles;
    n_int = A.n_int;
    nl = A.nl;
    L = A.L;
    site0 = (blk - tree * A.tiles) * SPW;
    leaf_base = (size_t)tree * nl * L;
    rows_base = (size_t)tree * n_int * L;
    site_base = (size_t)tree * L;
    steps = A.steps + (size_t)tree * n_int * 4;
  }
  const int site = site0 + grp;
  const bool active = grp < SPW && grp < in_item && site < L;
  const float a = A.a, bcoef = A.bcoef;

  float* X = lds;
  float* tab = lds + kXchg;                       // T[code][i]
  float* ctab = tab + wide_col_table_offset(G, Q);  // G > 4: lane columns of C / K
  WCoef<G> cf = cf_in;
  cf.cl = ctab + (w.i < G ? w.i : 0) * G;
  float* itab = tab + (Q + 1) * G;                // IK[code][i]
  float* slots = lds + kXchg + wide_tab_floats(G, Q);
  // fused factored softmin: each internal child's stabiliser md per site
  // group, kept from the forward for the adjoint ([n_int][SPW])
#ifdef TREX_DIAG_NO_KEEPMD
  constexpr bool KEEP_MD = false;
#else
  constexpr bool KEEP_MD = PHASE == 3 && MODE == kSoftK && G > 4;
#endif
  float* mdc = slots + (A.n_slots + 1) * kWave;
  int8_t* lleaf = reinterpret_cast<int8_t*>(mdc + (size_t)(A.nl - 1) * SPW);  // A.nl: max leaves

  // ---- prologue: leaf tables + leaf tile ----
  {
    const float sent = wmsg<G, MODE>(cf, X, w, a, bcoef, kSentinel);
    if (grp == 0) {
      for (int code = 0; code < Q; ++code) {
        const float cv = w.pad ? INFINITY : A.cost[w.i * Q + code];
        tab[code * G + w.i] = cv;
        if constexpr (MODE == kSoftK) itab[code * G + w.i] = w.pad ? 0.0f : fast_exp2((cv - cf.cmin) * a);
      }
      tab[Q * G + w.i] = sent;
      if constexpr (!SYM) fill_col_table<G, MODE>(ctab, A.cost, Q, w.i, cf.cmin, a);
    }
    const int8_t* lv = A.leaves + leaf_base;
    for (int t = lane; t < nl * SPW; t += kWave) {
      const int leaf = t / SPW;
      const int g = t - leaf * SPW;
      const int s = site0 + g;
      int code = (g < in_item && s < L) ? (int)lv[(size_t)leaf * L + s] : Q;
      code = ((unsigned)code < (unsigned)Q) ? code : Q;
      lleaf[t] = (int8_t)code;
    }
    wave_sync();
  }

  const cptr<int> prog = as_const(steps);
  const uint32_t rowbytes = (uint32_t)L * Q * 4;
  const uint32_t treebytes = (uint32_t)n_int * rowbytes;
  const rsrc_t rdp = make_rsrc(A.dp + rows_base * Q, treebytes);
  // inactive sites and padded states address past the buffer: stores drop, loads give 0
  const int voff = (active && !w.pad) ? (site * Q + w.i) * 4 : 0x7FFFFFF0;
  const int lgrp = grp < SPW ? grp : 0;

  float dv = 0.0f;
  if constexpr (FWD) {
    float prev = 0.0f;  // previous step's D (register bypass, kChildPrev)
    I4 nxt = load_step(prog, 0);
    for (int k = 0; k < n_int; ++k) {
      const I4 stp = nxt;
      if (k + 1 < n_int) nxt = load_step(prog, k + 1);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int desc = c == 0 ? stp.y : stp.z;
        const int kind = (desc >> 24) & 3;
        float m;
        if (kind == kKindLeaf) {
          const int code = lleaf[(desc & 0xFFFF) * SPW + lgrp];
          if constexpr (LFAST) {
            m = tab[code * G + w.i];
          } else {
            m = wmsg<G, MODE>(cf, X, w, a, bcoef, code == w.i ? 0.0f : kSentinel);
          }
        } else if (kind == kKindInt) {
          const float D = (desc & kChildPrev) ? prev : slots[((desc >> 16) & 0xFF) * kWave + lane];
          if constexpr (KEEP_MD) {
            float mdv;
            m = wmsg<G, MODE>(cf, X, w, a, bcoef, D, &mdv);
            if (w.i == 0) mdc[(desc & 0xFFFF) * SPW + lgrp] = mdv;
          } else {
            m = wmsg<G, MODE>(cf, X, w, a, bcoef, D);
          }
        } else {
          m = tab[Q * G + w.i];
        }
        dv = (c == 0) ? m : dv + m;
      }
      const int row = stp.x & 0xFFFF;
      const int oslot = (stp.x >> 16) & 0xFF;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dv), rdp, voff, row * rowbytes, 0);
      if (!(stp.w & kStepToNext) && oslot != 0xFF) slots[oslot * kWave + lane] = dv;
      prev = dv;
    }
  } else {
    dv = __uint_as_float(
        __builtin_amdgcn_raw_buffer_load_b32(rdp, voff, (n_int - 1) * rowbytes, 0));
  }

  // ---- root: score + cotangent (sankoff.py:187) ----
  float groot, score;
  {
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
  }
  const bool leader = active && w.i == 0;
  if constexpr (FWD) {
    if (leader && A.site_score) A.site_score[site_base + site] = score;
    const double tot = wave_sum(leader ? (double)score : 0.0);
    if (lane == 0) A.part_tree[blk] = tot;
  }

  if constexpr (BWD) {
    float acc[G];
#pragma unroll
    for (int j = 0; j < G; ++j) acc[j] = 0.0f;
    const float dscale = A.dts ? as_const(A.dts)[tree] : 1.0f;
    slots[A.n_slots * kWave + lane] = active ? groot * dscale : 0.0f;
    const bool want_marg = A.marg != nullptr;
    const rsrc_t rmg = make_rsrc(want_marg ? A.marg + rows_base * Q : A.dp, treebytes);
    const bool want_anc = A.anc != nullptr;
    int8_t* at = want_anc ? A.anc + rows_base + site : nullptr;

    // the next step's internal-child DP values are loaded one step ahead
    float nd[2] = {0.0f, 0.0f};
    I4 nstp = load_step(prog, n_int - 1);
    auto prefetch = [&](const I4& s2) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int desc = c == 0 ? s2.y : s2.z;
        if (((desc >> 24) & 3) == kKindInt)
          nd[c] = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(rdp, voff, (desc & 0xFFFF) * rowbytes, 0));
      }
    };
    prefetch(nstp);
    float gnext = 0.0f;  // cotangent handed to the next reverse step (bypass)
    for (int k = n_int - 1; k >= 0; --k) {
      const I4 stp = nstp;
      const float cd0 = nd[0], cd1 = nd[1];
      if (k > 0) {
        nstp = load_step(prog, k - 1);
        prefetch(nstp);
      }
      if (stp.w & kStepUnreached) continue;
      const int row = stp.x & 0xFFFF;
      const float g = (stp.w & kStepToNext)
                          ? gnext
                          : slots[((stp.w & kStepRoot) ? A.n_slots : ((stp.x >> 16) & 0xFF)) * kWave + lane];
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
          if constexpr (LFAST) onehot = !__any(active && code == Q);
          if (onehot) {
            // exact leaf weights are one-hot: dC[i][code] += g_i (/ K[i][code])
            float t = g;
            // (code Q only at sites past L, whose cotangent is 0: IK has no row Q)
            if constexpr (MODE == kSoftK) t = code < Q ? g * itab[code * G + w.i] : 0.0f;
            if (w.pad) t = 0.0f;
            onehot_add<G, MODE>(acc, w.i, code, t);
          } else {
            (void)wadj<G, MODE, SYM>(cf, X, w, a, code == w.i ? 0.0f : kSentinel, g, acc);
          }
        } else if (kind == kKindInt) {
          float gc;
          if constexpr (KEEP_MD)
            gc = wadj_k_md<G, SYM>(cf, X, w, a, c == 0 ? cd0 : cd1, mdc[(desc & 0xFFFF) * SPW + lgrp], g,
                              acc);
          else
            gc = wadj<G, MODE, SYM>(cf, X, w, a, c == 0 ? cd0 : cd1, g, acc);
          if (desc & kChildPrev) {
            gnext = gc;
          } else {
            const int cslot = (desc >> 16) & 0xFF;
            if (desc & kStepAccumulate) gc += slots[cslot * kWave + lane];
            slots[cslot * kWave + lane] = gc;
          }
        } else {
          (void)wadj<G, MODE, SYM>(cf, X, w, a, kSentinel, g, acc);
        }
      }
    }

    // ---- per-wave dC partial: rows i summed over the wave's sites ----
    const int nb = A.nitems;
#pragma unroll
    for (int j = 0; j < G; ++j) {
      double v = (double)acc[j];
      if constexpr (MODE == kSoftK) v *= (double)cf.row[j];
      double s = v;  // group 0 sums the groups in order
#pragma unroll
      for (int gq = 1; gq < SPW; ++gq) s += __shfl(v, w.i + gq * G, kWave);
      const int col = acc_col<G, MODE>(w.i, j);
      if (grp == 0 && !w.pad && col < Q) A.part_dc[(size_t)(w.i * Q + col) * nb + blk] = s;
    }
  }
}

template <int G, int MODE, int PHASE, bool RAGGED, bool SYM = false>
__device__ __forceinline__ void wide_dispatch_leaf(const WArgs& A, const WCoef<G>& cf, float cmax,
                                                   float* lds) {
  const float range = cmax - cf.cmin;
  const bool lfast = (MODE != kHard) ? ((kSentinel - range) * A.a >= 64.0f) : (range < 99000.0f);
  // one work item per workgroup (a grid-stride loop here raised the fused
  // Q = 20 kernel's scratch 56 -> 560 B: SGPR spills into VGPR lanes)
  const int blk = blockIdx.x;
  if (lfast)
    wide_body<G, MODE, PHASE, true, SYM, RAGGED>(A, cf, lds, blk);
  else
    wide_body<G, MODE, PHASE, false, SYM, RAGGED>(A, cf, lds, blk);
}

#ifndef TREX_WIDE_MINW
#define TREX_WIDE_MINW 4
#endif
// Q = 20 (C3): 4 waves per SIMD (<= 128 VGPRs) for the adjoint-bearing
// kernels -- 3 334 waves of C3 then fit the chip in one round
template <int G, int PHASE>
constexpr int wide_min_blocks() { return (G == 20 && (PHASE & 2)) ? TREX_WIDE_MINW : 1; }

template <int G, bool SOFT, int PHASE, bool RAGGED = false>
__global__ __launch_bounds__(kWave, (wide_min_blocks<G, PHASE>())) void sankoff_wide_kernel(WArgs A) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (A.skip && __hip_atomic_load(A.skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int Q = A.Q;
  const int i = threadIdx.x % G;
  if constexpr (SOFT && G > 4 && G <= kSiteSQ) {
    if (A.site_flag) {
      // the gate first, from a lane-parallel pass over C (<= 7 loads per
      // lane): when the lane-per-site kernel takes the call every workgroup
      // exits after it
      float lmin = INFINITY, lmax = -INFINITY;
      for (int e = threadIdx.x; e < Q * Q; e += kWave) {
        const float c = A.cost[e];
        lmin = fminf(lmin, c);
        lmax = fmaxf(lmax, c);
      }
      const float gmin = uniform(wave_minf(lmin)), gmax = uniform(wave_maxf(lmax));
      const bool handled = site_takes_call(gmin, gmax, A.a);
      if (blockIdx.x == 0) site_gate_write(A.cost, Q, gmin, A.a, A.site_kg, A.site_flag, handled);
      if (handled) {
        // the first workgroups build the cherry tables below K (their
        // (kSiteSQ + 1) kSiteSQ scratch floats are carved from the dynamic
        // LDS, which wide_run sizes to hold them on gated launches)
        site_pair_tables(A.cost, Q, gmin, A.a, A.bcoef, A.site_kg - kSiteTabBytes / 4, lds);
        return;
      }
    }
  }
  float cmin, cmax;
  bool sym;
  cost_range<G>(A.cost, Q, i, cmin, cmax, &sym);
  if constexpr (!SOFT) {
    wide_dispatch_leaf<G, kHard, PHASE, RAGGED>(A, make_coefs<G, kHard>(A.cost, Q, i, cmin, A.a), cmax,
                                                lds);
  } else if (use_ktrick(cmin, cmax, A.a)) {
    // symmetric costs (C3's protein matrix; C = 1 - I): K's column i is row
    // i, a variant without the column registers
    if (G > 4 && sym)
      wide_dispatch_leaf<G, kSoftK, PHASE, RAGGED, G != 4>(
          A, make_coefs<G, kSoftK>(A.cost, Q, i, cmin, A.a), cmax, lds);
    else
      wide_dispatch_leaf<G, kSoftK, PHASE, RAGGED>(A, make_coefs<G, kSoftK>(A.cost, Q, i, cmin, A.a),
                                                   cmax, lds);
  } else {
    wide_dispatch_leaf<G, kSoftDirect, PHASE, RAGGED>(
        A, make_coefs<G, kSoftDirect>(A.cost, Q, i, cmin, A.a), cmax, lds);
  }
}

// fixed-order reduction of per-item partials (both Sankoff paths): blocks
// [0, B) = tree scores, blocks [B, B + Q*Q) = dC entries; bitwise
// reproducible, and no arrival counters, so launches replay in hipGraphs
// 1 024 threads per entry: C4's dC entries sum 80 896 item partials each
// (28 -> ~8 us at 256 threads)
constexpr int kReduceThreads = 1024;
__global__ __launch_bounds__(kReduceThreads) void wide_reduce_kernel(const double* __restrict__ part_tree,
                                                          const double* __restrict__ part_dc,
                                                          int B, int tiles, int Q2, int do_tree,
                                                          float* __restrict__ tree_score,
                                                          float* __restrict__ d_cost,
                                                          const int* __restrict__ first,
                                                          int first_stride, int items,
                                                          int first_scale, const int* mx_flag,
                                                          int mx_tiles) {
  __shared__ double red[kReduceThreads];
  const int b = blockIdx.x;
  if (mx_flag && __hip_atomic_load(mx_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
    // the lane-per-site kernel's partials (sankoff_site.hip): mx_tiles per tree,
    // its dC block right after its B * mx_tiles tree partials
    tiles = mx_tiles;
    part_dc = part_tree + (size_t)B * mx_tiles;
  }
  const double* src;
  int n;
  float* dst;
  if (do_tree && b < B) {
    if (first) {  // ragged: tree b owns items [first[b], first[b + 1])
      const int lo = first[(size_t)b * first_stride] * first_scale;
      const int hi = (b + 1 < B ? first[(size_t)(b + 1) * first_stride] : items) * first_scale;
      src = part_tree + lo;
      n = hi - lo;
    } else {
      src = part_tree + (size_t)b * tiles;
      n = tiles;
    }
    dst = tree_score + b;
  } else {
    const int q = b - (do_tree ? B : 0);
    const size_t nb = first ? (size_t)items * first_scale : (size_t)B * tiles;
    src = part_dc + (size_t)q * nb;
    n = (int)nb;
    dst = d_cost + q;
  }
  const double v = fixed_sum<kReduceThreads>(src, n, red, threadIdx.x);
  if (threadIdx.x == 0) *dst = (float)v;
}

// Two-level form of the same fixed-order reduction for large uniform grids
// (C4: 80 896 items per dC entry, where one 1 024-thread block per entry is a
// chain of ten dependent load rounds, 23 us).  Stage 1: blocks [0, Q2 * P)
// each sum one kChunk-item chunk of one dC entry and write the result IN
// PLACE over the chunk's first partial (only this block reads the chunk);
// the remaining blocks sum tree scores, one wave per tree.  Stage 2: one wave
// per dC entry sums its P chunk results.  Partials are rewritten by every
// Sankoff launch, so consuming them in place is safe.
constexpr int kChunk = 2048;
#ifndef TREX_REDUCE2_MIN  // items per dC entry above which the two-level form runs
#define TREX_REDUCE2_MIN (4 * kChunk)
#endif
constexpr int kStage1Threads = 256;
__global__ __launch_bounds__(kStage1Threads) void reduce_stage1_kernel(
    const double* __restrict__ part_tree, double* __restrict__ part_dc, int B, int tiles, int ndc,
    int P, int do_tree, float* __restrict__ tree_score) {
  __shared__ double red[kStage1Threads];
  const int b = blockIdx.x;
  const size_t nb = (size_t)B * tiles;
  if (b < ndc) {
    const int q = b / P, p = b - q * P;
    double* src = part_dc + (size_t)q * nb + (size_t)p * kChunk;
    const int n = (int)min((size_t)kChunk, nb - (size_t)p * kChunk);
    const double v = fixed_sum<kStage1Threads>(src, n, red, threadIdx.x);
    if (threadIdx.x == 0) *src = v;  // every thread's loads retired before fixed_sum's barriers
    return;
  }
  if (!do_tree) return;
  const int t = (b - ndc) * (kStage1Threads / kWave) + (int)(threadIdx.x / kWave);
  if (t >= B) return;
  const int lane = threadIdx.x & (kWave - 1);
  const double* src = part_tree + (size_t)t * tiles;
  double acc = 0.0;
  for (int k = lane; k < tiles; k += kWave) acc += src[k];
  acc = wave_sum_lane0(acc);
  if (lane == 0) tree_score[t] = (float)acc;
}

__global__ __launch_bounds__(kWave) void reduce_stage2_kernel(const double* __restrict__ part_dc,
                                                               int B, int tiles, int P,
                                                               float* __restrict__ d_cost) {
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  const double* src = part_dc + (size_t)q * ((size_t)B * tiles);
  double acc = 0.0;
  for (int p = lane; p < P; p += kWave) acc += src[(size_t)p * kChunk];
  acc = wave_sum_lane0(acc);
  if (lane == 0) d_cost[q] = (float)acc;
}

// trex-exact ancestral reconstruction on the site-major table
// (sankoff.py:166-185, 191-267): one lane per site, C in LDS
// trex-exact reconstruction for Q > 4 (sankoff.py:166-185, 191-267): one
// lane per site walks the host-simulated DFS order.  The DP row each step
// reads does not depend on any state, so the next step's row is loaded while
// this step's argmin runs (ping-pong registers, loop unrolled by two); the
// states written so far stay in LDS ([n_int][64] bytes per wave) for the
// children's parent lookups instead of a global store -> load round trip
// on the chain.
template <int MQ, bool RAGGED = false>  // MQ 32: Q <= 32; 64: codon alphabets
__global__ __launch_bounds__(kWave) void wide_backtrack_kernel(const int* __restrict__ bt,
                                                               const float* __restrict__ cost,
                                                               const float* __restrict__ dp,
                                                               int n_int, int L, int Q, int tiles,
                                                               int8_t* __restrict__ anc,
                                                               const int* __restrict__ rmeta = nullptr,
                                                               int B = 0, int items = 0,
                                                               int steps = 0) {
  extern __shared__ __attribute__((aligned(16))) float bl[];
  float* c = bl;                                                // [Q][Q]
  int8_t* sts = reinterpret_cast<int8_t*>(bl + MQ * MQ);        // [n_int][64]
  int tree, tile;
  size_t rows_base;
  if constexpr (RAGGED) {  // ragged plan: per-tree record, item table, steps, entries
    const int item = blockIdx.x;
    tree = as_const(rmeta + (size_t)B * kRaggedMeta)[item];
    const cptr<int> m = as_const(rmeta) + (size_t)tree * kRaggedMeta;
    n_int = m[1];
    L = m[3];
    tile = item - m[5];
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
  const cptr<int> prog = as_const(bt);
  const float* dpt = dp + rows_base * Q + (size_t)site * Q;
  int8_t* at = anc + rows_base + site;
  // rows are 16-B aligned when Q % 4 == 0 (site * Q * 4): dwordx4 loads, a
  // quarter of the address work of 4-byte loads at an 4Q-byte lane stride
  const bool vec = (Q & 3) == 0;
  auto load_row = [&](int k, float (&o)[MQ]) {
    const int x = (k < n_int) ? (prog[2 * k] & 0xFFFF) : 0;
    const float* d = dpt + (size_t)x * L * Q;
    if (vec) {
#pragma unroll
      for (int v = 0; v < MQ / 4; ++v) {
        const float4 w = (4 * v < Q) ? reinterpret_cast<const float4*>(d)[v]
                                     : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        o[4 * v] = w.x;
        o[4 * v + 1] = w.y;
        o[4 * v + 2] = w.z;
        o[4 * v + 3] = w.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < MQ; ++j) o[j] = (j < Q) ? d[j] : 0.0f;
    }
  };
  auto step = [&](int k, const float (&d)[MQ]) {
    const int ex = prog[2 * k], ey = prog[2 * k + 1];
    const int x = ex & 0xFFFF;
    const int kind = (ex >> 16) & 0xF;
    int out = 0;
    if (kind != kBtUnreached) {
      const bool sent = kind == kBtSentinel;
      if (kind == kBtRoot) {
        float bv = d[0];
#pragma unroll
        for (int j = 1; j < MQ; ++j) {
          if (j >= Q) break;
          const float v = d[j];
          if (v < bv) { bv = v; out = j; }
        }
      } else {
        // parent's state: LDS for uniform batches; ragged batches (no bound
        // on a tree's node count at launch) re-read this lane's own output
        const int sp = RAGGED ? (int)at[(size_t)ey * L] : (int)sts[ey * kWave + lane];
        const float* row = c + sp * Q;
        float bv = row[0] + (sent ? kSentinel : d[0]);
#pragma unroll
        for (int j = 1; j < MQ; ++j) {
          if (j >= Q) break;
          const float v = row[j] + (sent ? kSentinel : d[j]);
          if (v < bv) { bv = v; out = j; }
        }
      }
    }
    if constexpr (!RAGGED) sts[x * kWave + lane] = (int8_t)out;
    at[(size_t)x * L] = (int8_t)out;
  };
  float r0[MQ], r1[MQ];
  load_row(0, r0);
  for (int k = 0; k < n_int; k += 2) {
    load_row(k + 1, r1);
    step(k, r0);
    if (k + 1 >= n_int) break;
    load_row(k + 2, r0);
    step(k + 1, r1);
  }
}

// Q <= 32, uniform batches: LPS = 8 (default) or 4 lanes per site (8 / 16
// sites per wave).  Lane q of a site scans states [q * ch, q * ch + ch), ch
// = ceil(Q / LPS), with trex's strict-< scan, and the site's lanes combine
// (smaller value, then lower index) by DPP -- the first-index argmin of
// sankoff.py:177-183, bit for bit.  8x the waves of the one-lane-per-site
// kernel (C3: 1 250 instead of 157) and an eighth of its serial compare
// chain per step; the parent states stay in LDS ([n_int][sites] bytes), the
// next rows are prefetched four steps ahead (read as dwords: a wave's sites
// are one contiguous span of each row)
// partner lane for combine level m of a site's LPS lanes: quad xor 1, xor 2,
// then the 8-lane half-row mirror (i <-> 7 - i: after the quad levels any
// cross-quad pairing completes the reduction, the combine being symmetric)
template <int M>
__device__ __forceinline__ int bt_partner(int v) {
  constexpr int ctrl = M == 1 ? 0xB1 : M == 2 ? 0x4E : 0x141;
  return __builtin_amdgcn_update_dpp(0, v, ctrl, 0xF, 0xF, true);
}
template <int LPS>  // lanes per site: 4 or 8
__global__ __launch_bounds__(kWave) void wide_backtrack4_kernel(const int* __restrict__ bt,
                                                                const float* __restrict__ cost,
                                                                const float* __restrict__ dp,
                                                                int n_int, int L, int Q, int tiles,
                                                                int8_t* __restrict__ anc) {
  constexpr int kBtCh = 32 / LPS;  // max states per lane (Q <= 32)
  constexpr int SPW = kWave / LPS;  // sites per wave
  extern __shared__ __attribute__((aligned(16))) float bl[];
  float* c = bl;                                          // [Q][Q] (32 x 32 reserved)
  int8_t* sts = reinterpret_cast<int8_t*>(bl + 32 * 32);  // [n_int][SPW]
  const int tree = blockIdx.x / tiles;
  const int tile = blockIdx.x - tree * tiles;
  const size_t rows_base = (size_t)tree * n_int * L;
  const int lane = threadIdx.x;
  for (int t = lane; t < 32 * 32; t += kWave) c[t] = t < Q * Q ? cost[t] : 0.0f;
  __syncthreads();
  const int sg = lane / LPS, q = lane % LPS;
  const int site = tile * SPW + sg;
  const bool live = site < L;  // no early exit: the quad combine needs every lane
  const int ch = (Q + LPS - 1) / LPS;
  const int j0 = q * ch;
  const cptr<int> prog = as_const(bt) + (size_t)tree * n_int * 2;
  const uint32_t rowbytes = (uint32_t)L * Q * 4;
  const rsrc_t rdp = make_rsrc(dp + rows_base * Q, (uint32_t)n_int * rowbytes);
  // lane offsets of its states; invalid states / dead sites read nothing
  int voff[kBtCh];
#pragma unroll
  for (int t = 0; t < kBtCh; ++t)
    voff[t] = (live && t < ch && j0 + t < Q) ? (site * Q + j0 + t) * 4 : 0x7FFFFFF0;
  int8_t* at = anc + rows_base + (live ? site : 0);
  auto load_row = [&](int k, float (&o)[kBtCh]) {
    const int x = (k < n_int) ? (prog[2 * k] & 0xFFFF) : 0;
#pragma unroll
    for (int t = 0; t < kBtCh; ++t)
      o[t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rdp, voff[t], x * rowbytes, 0));
  };
  auto step = [&](int k, const float (&d)[kBtCh]) {
    const int ex = prog[2 * k], ey = prog[2 * k + 1];
    const int x = ex & 0xFFFF;
    const int kind = (ex >> 16) & 0xF;
    int out = 0;
    if (kind != kBtUnreached) {
      const bool sent = kind == kBtSentinel;
      const bool root = kind == kBtRoot;
      const int sp = root ? 0 : (int)sts[ey * SPW + sg];
      const float* row = c + sp * Q + j0;
      float bv = INFINITY;
      int bi = j0;
#pragma unroll
      for (int t = 0; t < kBtCh; ++t) {
        const bool ok = t < ch && j0 + t < Q;
        const float dv = sent ? kSentinel : d[t];
        const float v = ok ? (root ? dv : row[t] + dv) : INFINITY;
        if (v < bv) { bv = v; bi = j0 + t; }
      }
      auto combine = [&](float ov, int oi) {
        if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      };
      combine(__int_as_float(bt_partner<1>(__float_as_int(bv))), bt_partner<1>(bi));
      combine(__int_as_float(bt_partner<2>(__float_as_int(bv))), bt_partner<2>(bi));
      if constexpr (LPS == 8)
        combine(__int_as_float(bt_partner<4>(__float_as_int(bv))), bt_partner<4>(bi));
      out = bi;
    }
    if (q == 0) {
      sts[x * SPW + sg] = (int8_t)out;
      if (live) at[(size_t)x * L] = (int8_t)out;
    }
  };
  float r0[kBtCh], r1[kBtCh], r2[kBtCh], r3[kBtCh];
  load_row(0, r0);
  load_row(1, r1);
  load_row(2, r2);
  load_row(3, r3);
  for (int k = 0; k < n_int; k += 4) {
    step(k, r0);
    load_row(k + 4, r0);
    if (k + 1 < n_int) step(k + 1, r1);
    load_row(k + 5, r1);
    if (k + 2 < n_int) step(k + 2, r2);
    load_row(k + 6, r2);
    if (k + 3 < n_int) step(k + 3, r3);
    load_row(k + 7, r3);
  }
}

template <int G, bool SOFT, bool RAGGED>
void launch_wide(int phase, int grid, size_t lds, hipStream_t st, const WArgs& A) {
  if (phase == 1)
    hipLaunchKernelGGL((sankoff_wide_kernel<G, SOFT, 1, RAGGED>), dim3(grid), dim3(kWave), lds, st, A);
  else if (phase == 2)
    hipLaunchKernelGGL((sankoff_wide_kernel<G, SOFT, 2, RAGGED>), dim3(grid), dim3(kWave), lds, st, A);
  else
    hipLaunchKernelGGL((sankoff_wide_kernel<G, SOFT, 3, RAGGED>), dim3(grid), dim3(kWave), lds, st, A);
}

template <int G, bool RAGGED = false>
void launch_wide_g(int phase, bool soft, int grid, size_t lds, hipStream_t st, const WArgs& A) {
  if (soft)
    launch_wide<G, true, RAGGED>(phase, grid, lds, st, A);
  else
    launch_wide<G, false, RAGGED>(phase, grid, lds, st, A);
}

}  // namespace

int wide_group(int Q) {
  if (Q <= 4) return 4;
  if (Q <= 8) return 8;
  if (Q <= 16) return 16;
  if (Q <= 20) return 20;
  if (Q <= 32) return 32;
  return 64;  // codon alphabets (61 / 64): one site per wave
}

int wide_tiles(int L, int Q) {
  const int spw = kWave / wide_group(Q);
  return (L + spw - 1) / spw;
}

size_t wide_lds_bytes(int n_slots, int nl, int ni, int Q) {
  const int G = wide_group(Q);
  const size_t b = (size_t)(kXchg + wide_tab_floats(G, Q) + (n_slots + 1) * kWave +
                            (size_t)ni * (kWave / G)) * 4 +
                   (size_t)nl * (kWave / G);
  return (b + 15) & ~(size_t)15;
}

int64_t wide_workspace_bytes(int B, int L, int Q) {
  const int64_t nb = (int64_t)B * wide_tiles(L, Q);
  // tail: staged-kernel counter (128 B) | cherry tables (36 KB) and K and
  // K^T (3.25 KB) for the lane-per-site kernel (sankoff_site.hip) | mode
  // flag (128 B)
  return nb * 8 * (1 + (int64_t)Q * Q) + 3584 + kSiteTabBytes;
}

int wide_run(const char* fn, const WideCall& c, bool reduce) {
  const int tiles = wide_tiles(c.L, c.Q);
  size_t lds = wide_lds_bytes(c.n_slots, c.nl, c.ni, c.Q);
  // a gated launch may build the site kernel's cherry tables in its LDS
  if (c.site_flag) lds = std::max(lds, (size_t)(kSiteSQ * kSiteSQ + kSiteSQ) * 4);
  if (lds > 65536) return set_error(TREX_E_UNSUPPORTED, "%s: LDS stack too deep", fn);
  if ((int64_t)c.B * tiles > 0x7FFFFFFF) return set_error(TREX_E_ARG, "%s: grid too large", fn);
  if ((int64_t)c.ni * c.L * c.Q * 4 > 0x7FFFFFF0LL)
    return set_error(TREX_E_UNSUPPORTED, "%s: one tree's DP table exceeds 2 GiB", fn);
  WArgs A;
  A.steps = c.steps;
  A.leaves = c.leaves;
  A.cost = c.cost;
  A.n_int = c.ni;
  A.nl = c.nl;
  A.L = c.L;
  A.tiles = tiles;
  A.B = c.B;
  A.n_slots = c.n_slots;
  A.Q = c.Q;
  A.a = c.a;
  A.bcoef = c.bcoef;
  A.hard_root = c.hard_root;
  A.dp = c.dp;
  A.site_score = c.site_score;
  A.dts = c.dts;
  A.marg = c.marg;
  A.anc = c.anc;
  A.rmeta = nullptr;
  A.ritem = nullptr;
  A.wpi = 0;
  A.skip = c.mx_flag;
  A.site_flag = c.site_flag;
  A.site_kg = c.site_kg;
  const int64_t nb = (int64_t)c.B * tiles;
  A.nitems = (int)nb;
  A.part_tree = static_cast<double*>(c.workspace);
  A.part_dc = A.part_tree + nb;
  hipStream_t st = (hipStream_t)c.stream;
  const int grid = (int)nb;
  switch (wide_group(c.Q)) {
    case 4: launch_wide_g<4>(c.phase, c.soft, grid, lds, st, A); break;
    case 8: launch_wide_g<8>(c.phase, c.soft, grid, lds, st, A); break;
    case 16: launch_wide_g<16>(c.phase, c.soft, grid, lds, st, A); break;
    case 20: launch_wide_g<20>(c.phase, c.soft, grid, lds, st, A); break;
    case 32: launch_wide_g<32>(c.phase, c.soft, grid, lds, st, A); break;
    default: launch_wide_g<64>(c.phase, c.soft, grid, lds, st, A); break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  if (!reduce) return TREX_OK;
  return partial_reduce(fn, A.part_tree, A.part_dc, c.B, tiles, c.Q, c.phase, c.tree_score,
                        c.d_cost, c.stream, nullptr, 0, 0, 1, c.mx_flag, c.mx_tiles);
}

// waves per 64-site ragged item: ceil(64 / sites per wave)
int wide_ragged_wpi(int Q) {
  const int spw = kWave / wide_group(Q);
  return (kWave + spw - 1) / spw;
}

int64_t wide_ragged_workspace_bytes(int64_t items, int Q) {
  return items * wide_ragged_wpi(Q) * 8 * (1 + (int64_t)Q * Q) + 256;
}

int wide_ragged_run(const char* fn, const WideCall& c, const int* rmeta, const int* ritem,
                    int64_t items) {
  const int wpi = wide_ragged_wpi(c.Q);
  const size_t lds = wide_lds_bytes(c.n_slots, c.nl, c.nl - 1, c.Q);
  if (lds > 65536) return set_error(TREX_E_UNSUPPORTED, "%s: LDS stack too deep", fn);
  if (items * wpi > 0x7FFFFFFF) return set_error(TREX_E_ARG, "%s: grid too large", fn);
  WArgs A;
  A.steps = c.steps;
  A.leaves = c.leaves;
  A.cost = c.cost;
  A.n_int = 0;
  A.nl = c.nl;  // max leaves (LDS leaf tile, stabiliser rows)
  A.L = 0;
  A.tiles = 0;
  A.B = c.B;
  A.n_slots = c.n_slots;
  A.Q = c.Q;
  A.a = c.a;
  A.bcoef = c.bcoef;
  A.hard_root = c.hard_root;
  A.dp = c.dp;
  A.site_score = c.site_score;
  A.dts = c.dts;
  A.marg = c.marg;
  A.anc = c.anc;
  A.rmeta = rmeta;
  A.ritem = ritem;
  A.wpi = wpi;
  A.skip = nullptr;  // ragged batches never run the matrix-core kernel
  const int grid = (int)(items * wpi);
  A.nitems = grid;
  A.part_tree = static_cast<double*>(c.workspace);
  A.part_dc = A.part_tree + grid;
  hipStream_t st = (hipStream_t)c.stream;
  switch (wide_group(c.Q)) {
    case 8: launch_wide_g<8, true>(c.phase, c.soft, grid, lds, st, A); break;
    case 16: launch_wide_g<16, true>(c.phase, c.soft, grid, lds, st, A); break;
    case 20: launch_wide_g<20, true>(c.phase, c.soft, grid, lds, st, A); break;
    case 32: launch_wide_g<32, true>(c.phase, c.soft, grid, lds, st, A); break;
    default: launch_wide_g<64, true>(c.phase, c.soft, grid, lds, st, A); break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return partial_reduce(fn, A.part_tree, A.part_dc, c.B, 0, c.Q, c.phase, c.tree_score, c.d_cost,
                        c.stream, rmeta + 5, kRaggedMeta, (int)items, wpi);
}

int partial_reduce(const char* fn, const double* part_tree, const double* part_dc, int B,
                   int tiles, int Q, int phase, float* tree_score, float* d_cost, void* stream,
                   const int* first, int first_stride, int items, int first_scale,
                   const int* mx_flag, int mx_tiles) {
  const bool do_tree = (phase & 1) != 0;
  const bool do_dc = (phase & 2) != 0;
  const int64_t nb = (int64_t)B * tiles;
  if (!first && !mx_flag && do_dc && nb > TREX_REDUCE2_MIN) {
    const int P = (int)((nb + kChunk - 1) / kChunk);
    const int ndc = Q * Q * P;
    const int tblocks = do_tree ? (B + kStage1Threads / kWave - 1) / (kStage1Threads / kWave) : 0;
    hipLaunchKernelGGL(reduce_stage1_kernel, dim3(ndc + tblocks), dim3(kStage1Threads), 0,
                       (hipStream_t)stream, part_tree, const_cast<double*>(part_dc), B, tiles, ndc,
                       P, do_tree ? 1 : 0, tree_score);
    hipLaunchKernelGGL(reduce_stage2_kernel, dim3(Q * Q), dim3(kWave), 0, (hipStream_t)stream,
                       part_dc, B, tiles, P, d_cost);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
    return TREX_OK;
  }
  const int rgrid = (do_tree ? B : 0) + (do_dc ? Q * Q : 0);
  hipLaunchKernelGGL(wide_reduce_kernel, dim3(rgrid), dim3(kReduceThreads), 0, (hipStream_t)stream,
                     part_tree, part_dc, B, tiles, Q * Q, do_tree ? 1 : 0, tree_score, d_cost,
                     first, first_stride, items, first_scale, mx_flag, mx_tiles);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

int wide_ragged_backtrack(const int32_t* rmeta, int B, int64_t items, int64_t steps,
                          const float* cost, const float* dp, int Q, int8_t* anc, void* stream) {
  const int mq = Q <= 32 ? 32 : 64;
  const size_t lds = (size_t)mq * mq * 4;
  if (mq == 32)
    hipLaunchKernelGGL((wide_backtrack_kernel<32, true>), dim3((int)items), dim3(kWave), lds,
                       (hipStream_t)stream, nullptr, cost, dp, 0, 0, Q, 0, anc, rmeta, B,
                       (int)items, (int)steps);
  else
    hipLaunchKernelGGL((wide_backtrack_kernel<64, true>), dim3((int)items), dim3(kWave), lds,
                       (hipStream_t)stream, nullptr, cost, dp, 0, 0, Q, 0, anc, rmeta, B,
                       (int)items, (int)steps);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_error(TREX_E_HIP, "trex_sankoff_ragged_backtrack: %s", hipGetErrorString(e));
  return TREX_OK;
}

int wide_backtrack(const int32_t* bt, const float* cost, const float* dp, int B, int L, int ni,
                   int Q, int8_t* anc, void* stream) {
  // TREX_BT4=0 forces the one-lane-per-site kernel (live for codons, ragged
  // batches and trees too deep for the split kernel's LDS; the tests run it
  // on Q <= 32 too).  8 lanes per site for Q > 4; Q <= 4 (one state per lane): 4
  const char* e4 = std::getenv("TREX_BT4");
  const int lps = Q <= 4 ? 4 : 8;
  if (Q <= 32 && !(e4 && e4[0] == '0') && (int64_t)ni * L * Q * 4 <= 0x7FFFFFF0LL &&
      32 * 32 * 4 + (size_t)ni * (kWave / lps) <= 65536) {
    const int spw = kWave / lps;
    const int tiles4 = (L + spw - 1) / spw;
    const size_t lds4 = 32 * 32 * 4 + (size_t)ni * spw;
    if (lps == 8)
      hipLaunchKernelGGL(wide_backtrack4_kernel<8>, dim3(B * tiles4), dim3(kWave), lds4,
                         (hipStream_t)stream, bt, cost, dp, ni, L, Q, tiles4, anc);
    else
      hipLaunchKernelGGL(wide_backtrack4_kernel<4>, dim3(B * tiles4), dim3(kWave), lds4,
                         (hipStream_t)stream, bt, cost, dp, ni, L, Q, tiles4, anc);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
      return set_error(TREX_E_HIP, "trex_sankoff_backtrack: %s", hipGetErrorString(e));
    return TREX_OK;
  }
  const int tiles = (L + kWave - 1) / kWave;
  const int mq = Q <= 32 ? 32 : 64;
  const size_t lds = (size_t)mq * mq * 4 + (size_t)ni * kWave;
  if (lds > 160 * 1024)
    return set_error(TREX_E_UNSUPPORTED, "trex_sankoff_backtrack: %d internal nodes", ni);
  auto go = [&](auto kernel) {
    if (lds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kernel, dim3(B * tiles), dim3(kWave), lds, (hipStream_t)stream, bt, cost, dp,
                       ni, L, Q, tiles, anc, (const int*)nullptr, 0, 0, 0);
  };
  if (mq == 32)
    go(wide_backtrack_kernel<32, false>);
  else
    go(wide_backtrack_kernel<64, false>);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_error(TREX_E_HIP, "trex_sankoff_backtrack: %s", hipGetErrorString(e));
  return TREX_OK;
}

}  // namespace trex
