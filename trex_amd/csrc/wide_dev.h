// Device helpers of the state-parallel Sankoff kernels (sankoff_wide.hip:
// one wave per work item; sankoff_staged.hip: one workgroup of waves per
// item, nodes spread over the waves): a group of G lanes owns one site, lane
// i of the group owns parent state i (trex src/trex/sankoff.py run_dp :24-94
// semantics, build-defined softmin adjoint).
#pragma once

#include <hip/hip_runtime.h>

#include "sankoff_dev.h"

namespace trex {
namespace {

// 4 exchange buffers [4][64] floats per wave; leaf message table T[Q + 1][G]
// (row Q = message of the all-1e5 row) and IK[Q][G] = 1 / K[i][code]
constexpr int kXchg = 4 * kWave;

// leaf message table T[Q + 1][G], IK[Q][G], and for G > 4 the per-lane
// column table CT[G][G] (CT[i][j] = column i of C / K at row j)
__host__ __device__ constexpr int wide_tab_floats(int G, int Q) {
  return (2 * Q + 1) * G + (G > 4 ? G * G : 0);
}
__host__ __device__ constexpr int wide_col_table_offset(int G, int Q) { return (2 * Q + 1) * G; }


__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

template <int K_>
__device__ __forceinline__ float quad_bcast(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), K_ * 0x55, 0xF, 0xF, false));
}

// every lane publishes v; each lane gets the G values of its own group.
// G = 4 (Q <= 4 on small grids): the group is a DPP quad -- four quad
// broadcasts, no LDS round trip
template <int G>
__device__ __forceinline__ void xchg(float* x, int lane, int gbase, float v, float (&o)[G]) {
  if constexpr (G == 4) {
    (void)x;
    (void)lane;
    (void)gbase;
    o[0] = quad_bcast<0>(v);
    o[1] = quad_bcast<1>(v);
    o[2] = quad_bcast<2>(v);
    o[3] = quad_bcast<3>(v);
    return;
  }
  x[lane] = v;
  wave_sync();
#pragma unroll
  for (int t = 0; t < G / 4; ++t) {
    const float4 w = reinterpret_cast<const float4*>(x + gbase)[t];
    o[4 * t] = w.x;
    o[4 * t + 1] = w.y;
    o[4 * t + 2] = w.z;
    o[4 * t + 3] = w.w;
  }
  wave_sync();
}

__device__ __forceinline__ float wave_minf(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, kWave));
  return v;
}
__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// row[j] / col[j]: C[i][j] / C[j][i] (hard, direct) or K[i][j] / K[j][i] (K mode)
template <int G>
struct WCoef {
  float row[G];
  float col[G];        // G = 4 only (G > 4: the LDS table cl, or row when symmetric)
  const float* cl;     // G > 4: this lane's column of C / K in LDS (wide_col_table)
  float cmin;
};

// G = 4, factored softmin (C2 / C4-shaped DNA on small grids): the quad's
// exchanges are xor quad-permutations applied as DPP operands, and lane i
// keeps its coefficients and dC accumulators in xor order: row[p] =
// K[i][i^p], col[p] = K[i^p][i], acc[p] = dC[i][i^p] (xor_perm_coefs at
// kernel start; acc_col maps back).  No broadcast copies of the quad.
template <int G, int MODE>
__host__ __device__ constexpr bool xor_perm() {
  return G == 4 && MODE == kSoftK;
}
template <int G, int MODE>
__device__ __forceinline__ int acc_col(int i, int j) {
  if constexpr (xor_perm<G, MODE>()) return i ^ j;
  return j;
}
template <int P>
__device__ __forceinline__ float qx(float v) {  // lane i of a quad gets v of lane i ^ P
  constexpr int ctrl = P == 1 ? 0xB1 : P == 2 ? 0x4E : 0x1B;
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, true));
}
__device__ __forceinline__ float sel4(const float (&v)[4], int k) {
  return k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3];
}

struct WLane {
  int lane, i, gbase;
  bool pad;  // state i >= Q
};

// wave-uniform min / max over the cost matrix (every lane scans its row)
template <int G>
__device__ __forceinline__ void cost_range(const float* cost, int Q, int i, float& cmin,
                                           float& cmax, bool* sym = nullptr) {
  float lmin = INFINITY, lmax = -INFINITY;
  bool s = true;
  if (i < Q) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      if (j < Q) {
        const float c = cost[i * Q + j];
        lmin = fminf(lmin, c);
        lmax = fmaxf(lmax, c);
        s = s && c == cost[j * Q + i];
      }
    }
  }
  cmin = uniform(wave_minf(lmin));
  cmax = uniform(wave_maxf(lmax));
  if (sym) *sym = __all(s);
}

// ---- gate of the lane-per-site kernel (sankoff_site.hip, 4 < Q <= 20) ----
// It takes a soft call when the factored softmin applies and the 1e5
// sentinel dominates (exact leaf messages); it reads K = exp(-(C - cmin) /
// tau) [20][20] and K^T with scalar loads.  The state-parallel kernel,
// launched first, decides this on every workgroup from the cost matrix;
// its workgroup 0 writes K, K^T and the flag for the site kernel and the
// reduce launched behind it (no separate prologue launch).
constexpr int kSiteSQ = 20;
__device__ __forceinline__ bool site_takes_call(float cmin, float cmax, float a) {
  return use_ktrick(cmin, cmax, a) && (kSentinel - (cmax - cmin)) * a >= 64.0f;
}
__device__ __forceinline__ void site_gate_write(const float* cost, int Q, float cmin, float a,
                                                float* kg, int* flag, bool handled) {
  const int lane = threadIdx.x & (kWave - 1);
  for (int e = lane; e < kSiteSQ * kSiteSQ; e += kWave) {
    const int i = e / kSiteSQ, j = e - i * kSiteSQ;
    const float kv = (i < Q && j < Q) ? fast_exp2((cmin - cost[i * Q + j]) * a) : 0.0f;
    kg[e] = kv;                                  // K [i][j]
    kg[kSiteSQ * kSiteSQ + j * kSiteSQ + i] = kv;  // K^T [j][i]
  }
  if (lane == 0) flag[0] = handled ? 1 : 0;
}

// ---- cherry tables of the lane-per-site kernel ----
// A cherry (an internal row whose two children are leaves or 1e5 rows) has
// D = T[c0] + T[c1], with T the leaf-message table (T[c][i] = C[i][c],
// T[Q] the all-1e5 row's message): one of (Q + 1)(Q + 2) / 2 vectors.  The
// gate builds, per unordered code pair, the cherry's forward message to its
// parent (TM) and its softmin row sums s = K u (TS), with the site kernel's
// arithmetic step for step (bitwise what it would compute per lane), so the
// site kernel replaces a cherry's K mat-vec -- both of the forward's and one
// of the adjoint's -- by a table row.  Workspace: TM [pairs][20] | TS
// [pairs][20] just below K / K^T.
constexpr int kSitePairs = (kSiteSQ + 1) * (kSiteSQ + 2) / 2;
constexpr int kSiteTabBytes = (2 * kSitePairs * kSiteSQ * 4 + 127) / 128 * 128;
__device__ __forceinline__ int site_pair(int c0, int c1) {
  const int lo = c0 < c1 ? c0 : c1, hi = c0 < c1 ? c1 : c0;
  return hi * (hi + 1) / 2 + lo;
}
// one (pair, state) entry per thread: the workgroups of the gate share the
// (Q + 1)(Q + 2) / 2 * 20 entries (64 per workgroup and round, 73
// workgroups at Q = 20), each thread recomputing its pair's D and u (20
// values) and its own row sum s_i -- a few hundred instructions, so the
// gate launch the site kernel waits on stays short.  kl: [kSiteSQ *
// kSiteSQ + kSiteSQ] floats of LDS (this workgroup's K, then T[Q])
__device__ __forceinline__ void site_pair_tables(const float* cost, int Q, float cmin, float a,
                                                 float bcoef, float* tm, float* kl) {
  const int lane = threadIdx.x & (kWave - 1);
  constexpr int kEntries = kSitePairs * kSiteSQ;
  if ((int)blockIdx.x * kWave >= kEntries) return;
  for (int e = lane; e < kSiteSQ * kSiteSQ; e += kWave) {
    const int i = e / kSiteSQ, j = e - i * kSiteSQ;
    kl[e] = (i < Q && j < Q) ? fast_exp2((cmin - cost[i * Q + j]) * a) : 0.0f;
  }
  __syncthreads();
  float* tq = kl + kSiteSQ * kSiteSQ;  // T[Q][i]: the all-1e5 row's message
  if (lane < kSiteSQ) {
    float sk = 0.0f;
    for (int j = 0; j < Q; ++j) sk += kl[lane * kSiteSQ + j];
    tq[lane] = lane < Q ? fmaf(-bcoef, fast_log2(sk), kSentinel + cmin) : 0.0f;
  }
  __syncthreads();
  float* ts = tm + kSitePairs * kSiteSQ;
  for (int t = (int)blockIdx.x * kWave + lane; t < kEntries; t += (int)gridDim.x * kWave) {
    const int p = t / kSiteSQ, i = t - p * kSiteSQ;
    int hi = 0;
    while ((hi + 1) * (hi + 2) / 2 <= p) ++hi;
    const int lo = p - hi * (hi + 1) / 2;
    if (hi > Q) continue;  // codes are 0..Q
    // T[c][j] as the site kernel's prologue builds it (sankoff_site.hip)
    auto trow = [&](int code, int j) -> float {
      return j >= Q ? 0.0f : code < Q ? cost[j * Q + code] : tq[j];
    };
    float d[kSiteSQ];
#pragma unroll
    for (int j = 0; j < kSiteSQ; ++j) d[j] = trow(lo, j) + trow(hi, j);
    float md = d[0];
#pragma unroll
    for (int j = 1; j < kSiteSQ; ++j) md = j < Q ? fminf(md, d[j]) : md;
    const float mda = md * a;
    float sv = 0.0f;
#pragma unroll
    for (int j = 0; j < kSiteSQ; ++j)
      if (j < Q) sv = fmaf(kl[i * kSiteSQ + j], fast_exp2(fmaf(-d[j], a, mda)), sv);
    sv = i < Q ? sv : 1.0f;
    ts[t] = sv;
    tm[t] = i < Q ? fmaf(-bcoef, fast_log2(sv), md + cmin) : 0.0f;
  }
}

template <int G>
__device__ __forceinline__ void xor_perm_coefs(WCoef<G>& cf, int i);

// lane i's row / column of C (kHard, kSoftDirect) or of K = exp(-(C - cmin) /
// tau) (kSoftK; xor order for G = 4).  Built inside each mode's branch so the
// modes' register lifetimes never overlap (one kernel holds all of them)
template <int G, int MODE>
__device__ __forceinline__ WCoef<G> make_coefs(const float* cost, int Q, int i, float cmin,
                                               float a) {
  WCoef<G> cf;
  const bool pad = i >= Q;
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const bool ok = !pad && j < Q;
    const float r = ok ? cost[i * Q + j] : INFINITY;
    const float c = ok ? cost[j * Q + i] : INFINITY;
    if constexpr (MODE == kSoftK) {
      cf.row[j] = ok ? fast_exp2((cmin - r) * a) : 0.0f;
      cf.col[j] = (G == 4 && ok) ? fast_exp2((cmin - c) * a) : 0.0f;
    } else {
      cf.row[j] = r;
      cf.col[j] = G == 4 ? c : 0.0f;
    }
  }
  cf.cl = nullptr;
  cf.cmin = cmin;
  if constexpr (MODE == kSoftK) xor_perm_coefs<G>(cf, i);
  return cf;
}

template <int G>
__device__ __forceinline__ void xor_perm_coefs(WCoef<G>& cf, int i) {
  if constexpr (G == 4) {
    float r[4], c[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      r[p] = sel4(cf.row, i ^ p);
      c[p] = sel4(cf.col, i ^ p);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      cf.row[p] = r[p];
      cf.col[p] = c[p];
    }
  }
}

// message to parent state i:  min_j / smin_j (C[i][j] + D[j])   (sankoff.py:67-68)
template <int G, int MODE>
__device__ __forceinline__ float wmsg(const WCoef<G>& cf, float* X, const WLane& w, float a,
                                      float bcoef, float D, float* md_out = nullptr) {
  if constexpr (xor_perm<G, MODE>()) {
    (void)X;
    const float Dv = w.pad ? INFINITY : D;
    float md = fminf(Dv, qx<1>(Dv));
    md = fminf(md, qx<2>(md));
    const float u = w.pad ? 0.0f : fast_exp2((md - D) * a);
    float s = cf.row[0] * u;
    s = fmaf(cf.row[1], qx<1>(u), s);
    s = fmaf(cf.row[2], qx<2>(u), s);
    s = fmaf(cf.row[3], qx<3>(u), s);
    return fmaf(-bcoef, fast_log2(s), md + cf.cmin);
  }
  float d[G];
  xchg<G>(X, w.lane, w.gbase, w.pad ? INFINITY : D, d);
  if constexpr (MODE == kHard) {
    float v = cf.row[0] + d[0];
#pragma unroll
    for (int j = 1; j < G; ++j) v = fminf(v, cf.row[j] + d[j]);
    return v;
  } else if constexpr (MODE == kSoftK) {
    float md = d[0];
#pragma unroll
    for (int j = 1; j < G; ++j) md = fminf(md, d[j]);
    if (md_out) *md_out = md;
    const float u = w.pad ? 0.0f : fast_exp2((md - D) * a);
    float uu[G];
    xchg<G>(X + kWave, w.lane, w.gbase, u, uu);
    return fmaf(-bcoef, fast_log2(kdot<G>(cf.row, uu)), md + cf.cmin);
  } else {
    float x[G];
    float mn = INFINITY;
#pragma unroll
    for (int j = 0; j < G; ++j) {
      x[j] = cf.row[j] + d[j];
      mn = fminf(mn, x[j]);
    }
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < G; ++j) s += fast_exp2((mn - x[j]) * a);
    return fmaf(-bcoef, fast_log2(s), mn);
  }
}

// adjoint of one child message: acc[j] += g_i w_ij (row i of dC; in the K
// form the K[i][j] factor is applied once at the end); returns the child's
// cotangent for state i:  gc_i = sum_p g_p w_pi
// lane i's column of C (kHard, kSoftDirect) / K (kSoftK) into the LDS
// table at ct (G > 4; called by the lanes of one group)
template <int G, int MODE>
__device__ __forceinline__ void fill_col_table(float* ct, const float* cost, int Q, int i,
                                               float cmin, float a) {
  if constexpr (G > 4) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const bool ok = i < Q && j < Q;
      const float c = ok ? cost[j * Q + i] : INFINITY;
      ct[i * G + j] = MODE == kSoftK ? (ok ? fast_exp2((cmin - c) * a) : 0.0f) : c;
    }
  }
}
template <int G, bool SYM>
__device__ __forceinline__ float ccol(const WCoef<G>& cf, int p) {
  if constexpr (SYM) return cf.row[p];
  else if constexpr (G == 4) return cf.col[p];
  else return cf.cl[p];
}
// sum_p column[p] * r[p], the LDS column streamed in float4 chunks
template <int G, bool SYM>
__device__ __forceinline__ float kdot_col(const WCoef<G>& cf, const float (&r)[G]) {
  if constexpr (SYM) {
    return kdot<G>(cf.row, r);
  } else if constexpr (G == 4) {
    return kdot<G>(cf.col, r);
  } else {
    f2 acc2 = pk(0.0f, 0.0f);
#pragma unroll
    for (int t = 0; t < G / 4; ++t) {
      const float4 v = reinterpret_cast<const float4*>(cf.cl)[t];
      acc2 = __builtin_elementwise_fma(pk(v.x, v.y), pk(r[4 * t], r[4 * t + 1]), acc2);
      acc2 = __builtin_elementwise_fma(pk(v.z, v.w), pk(r[4 * t + 2], r[4 * t + 3]), acc2);
    }
    return acc2.x + acc2.y;
  }
}

// SYM: the cost matrix is symmetric (so is K): column i of K is row i, and
// the column registers are never read (the compiler drops them)
template <int G, int MODE, bool SYM = false>
__device__ __forceinline__ float wadj(const WCoef<G>& cf, float* X, const WLane& w, float a,
                                      float D, float g, float (&acc)[G]) {
  if constexpr (xor_perm<G, MODE>()) {
    (void)X;
    const float Dv = w.pad ? INFINITY : D;
    float md = fminf(Dv, qx<1>(Dv));
    md = fminf(md, qx<2>(md));
    const float u = w.pad ? 0.0f : fast_exp2((md - D) * a);
    const float u1 = qx<1>(u), u2 = qx<2>(u), u3 = qx<3>(u);
    float s = cf.row[0] * u;
    s = fmaf(cf.row[1], u1, s);
    s = fmaf(cf.row[2], u2, s);
    s = fmaf(cf.row[3], u3, s);
    const float r = w.pad ? 0.0f : g * __builtin_amdgcn_rcpf(s);
    acc[0] = fmaf(r, u, acc[0]);
    acc[1] = fmaf(r, u1, acc[1]);
    acc[2] = fmaf(r, u2, acc[2]);
    acc[3] = fmaf(r, u3, acc[3]);
    // gc_i = u_i sum_q K[i^q][i] r_{i^q}
    float t = cf.col[0] * r;
    t = fmaf(cf.col[1], qx<1>(r), t);
    t = fmaf(cf.col[2], qx<2>(r), t);
    t = fmaf(cf.col[3], qx<3>(r), t);
    return u * t;
  }
  float d[G];
  xchg<G>(X, w.lane, w.gbase, w.pad ? INFINITY : D, d);
  float rr[G];
  if constexpr (MODE == kSoftK) {
    float md = d[0];
#pragma unroll
    for (int j = 1; j < G; ++j) md = fminf(md, d[j]);
    const float u = w.pad ? 0.0f : fast_exp2((md - D) * a);
    float uu[G];
    xchg<G>(X + kWave, w.lane, w.gbase, u, uu);
    const float r = w.pad ? 0.0f : g * __builtin_amdgcn_rcpf(kdot<G>(cf.row, uu));
    axpy<G>(acc, r, uu);
    xchg<G>(X + 2 * kWave, w.lane, w.gbase, r, rr);
    return u * kdot_col<G, SYM>(cf, rr);
  } else if constexpr (MODE == kHard) {
    float x[G];
    float mn = cf.row[0] + d[0];
    x[0] = mn;
#pragma unroll
    for (int j = 1; j < G; ++j) {
      x[j] = cf.row[j] + d[j];
      mn = fminf(mn, x[j]);
    }
    float cnt = 0.0f;
#pragma unroll
    for (int j = 0; j < G; ++j) cnt += (x[j] == mn) ? 1.0f : 0.0f;
    const float r = w.pad ? 0.0f : g / cnt;
#pragma unroll
    for (int j = 0; j < G; ++j) acc[j] += (x[j] == mn) ? r : 0.0f;
    float mm[G];
    xchg<G>(X + 2 * kWave, w.lane, w.gbase, r, rr);
    xchg<G>(X + 3 * kWave, w.lane, w.gbase, w.pad ? 0.0f : mn, mm);
    // parent p's x_{p i} = C[p][i] + D_i, bit-identical to lane p's x[i]
    float gc = 0.0f;
#pragma unroll
    for (int p = 0; p < G; ++p) gc += (ccol<G, SYM>(cf, p) + D == mm[p]) ? rr[p] : 0.0f;
    return gc;
  } else {
    // per-row stabilised softmin (rare: range(C)/tau > 40); computed in
    // place in d[] and, for G > 4, the parents' r / mn streamed from the
    // exchange buffers: this mode's transients set the register budget of
    // the whole kernel
    float mn = INFINITY;
#pragma unroll
    for (int j = 0; j < G; ++j) {
      d[j] = cf.row[j] + d[j];
      mn = fminf(mn, d[j]);
    }
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < G; ++j) {
      d[j] = fast_exp2((mn - d[j]) * a);
      s += d[j];
    }
    const float r = w.pad ? 0.0f : g * __builtin_amdgcn_rcpf(s);
    axpy<G>(acc, r, d);
    if constexpr (G > 4) {
      float* xr = X + 2 * kWave;
      float* xm = X + 3 * kWave;
      xr[w.lane] = r;
      xm[w.lane] = w.pad ? 0.0f : mn;
      wave_sync();
      float gc = 0.0f;
#pragma unroll
      for (int t = 0; t < G / 4; ++t) {
        const float4 rv = reinterpret_cast<const float4*>(xr + w.gbase)[t];
        const float4 mv = reinterpret_cast<const float4*>(xm + w.gbase)[t];
        gc += rv.x * fast_exp2((mv.x - (ccol<G, SYM>(cf, 4 * t) + D)) * a);
        gc += rv.y * fast_exp2((mv.y - (ccol<G, SYM>(cf, 4 * t + 1) + D)) * a);
        gc += rv.z * fast_exp2((mv.z - (ccol<G, SYM>(cf, 4 * t + 2) + D)) * a);
        gc += rv.w * fast_exp2((mv.w - (ccol<G, SYM>(cf, 4 * t + 3) + D)) * a);
      }
      wave_sync();
      return gc;
    }
    float mm[G];
    xchg<G>(X + 2 * kWave, w.lane, w.gbase, r, rr);
    xchg<G>(X + 3 * kWave, w.lane, w.gbase, w.pad ? 0.0f : mn, mm);
    float gc = 0.0f;
#pragma unroll
    for (int p = 0; p < G; ++p) gc += rr[p] * fast_exp2((mm[p] - (ccol<G, SYM>(cf, p) + D)) * a);
    return gc;
  }
}

// exact one-hot leaf weight: acc[slot of column code] += t.  G > 4: pairs
// of slots at once, one-hot(j) = clamp(1 - (code - j)^2) on packed FP32
// (exact for integer codes; clamp folded into the packed FMA) -- 1.5 VALU
// per slot instead of a compare, select and add
__device__ __forceinline__ f2 onehot2(f2 x) {
  f2 y;
  asm("v_pk_fma_f32 %0, %1, %1, 1.0 op_sel_hi:[1,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0] clamp"
      : "=v"(y)
      : "v"(x));
  return y;
}
template <int G, int MODE>
__device__ __forceinline__ void onehot_add(float (&acc)[G], int i, int code, float t) {
  if constexpr (G > 4 && G % 2 == 0) {
    const float f = (float)code;
#pragma unroll
    for (int j = 0; j < G; j += 2)
      pfma(acc[j], acc[j + 1], pk(t, t), onehot2(pk(f, f) - pk((float)j, (float)(j + 1))));
  } else {
#pragma unroll
    for (int j = 0; j < G; ++j) acc[j] += (code == acc_col<G, MODE>(i, j)) ? t : 0.0f;
  }
}

// first-index argmax of the group's values v (lane i holds state i; padded
// states pass -inf): the group max, then the lowest lane of the group that
// holds it from a wave ballot -- no G-step compare / select chain
template <int G>
__device__ __forceinline__ int group_argmax(float* X, const WLane& w, float v) {
  float gg[G];
  xchg<G>(X, w.lane, w.gbase, v, gg);
  float bv = gg[0];
#pragma unroll
  for (int j = 1; j < G; ++j) bv = fmaxf(bv, gg[j]);
  const unsigned long long hit = __ballot(!w.pad && v == bv);
  return __builtin_ctzll((hit >> w.gbase) | (1ull << 63));
}

// wadj for the factored softmin when the child's stabiliser md = min_j D[j]
// is already known (kept from the fused kernel's forward): no exchange of D
// and no G-way min -- the same arithmetic, bitwise the same result
template <int G, bool SYM = false>
__device__ __forceinline__ float wadj_k_md(const WCoef<G>& cf, float* X, const WLane& w, float a,
                                           float D, float md, float g, float (&acc)[G]) {
  // (min: sites past L read D = 0 in the adjoint, not their forward value;
  // exact no-op for real sites, md <= D)
  const float u = w.pad ? 0.0f : fast_exp2(fminf((md - D) * a, 0.0f));
  float uu[G];
  xchg<G>(X + kWave, w.lane, w.gbase, u, uu);
  const float r = w.pad ? 0.0f : g * __builtin_amdgcn_rcpf(kdot<G>(cf.row, uu));
  axpy<G>(acc, r, uu);
  float rr[G];
  xchg<G>(X + 2 * kWave, w.lane, w.gbase, r, rr);
  return u * kdot_col<G, SYM>(cf, rr);
}

// Fixed-order sum of n doubles by the NT threads of a block (red[NT] in
// LDS); the result is in thread 0's return value.  Eight independent
// accumulators keep eight loads in flight per thread; the association is
// fixed (bitwise reproducible).  Every thread of the block must call it.
template <int NT>
__device__ __forceinline__ double fixed_sum(const double* src, int n, double* red, int t) {
  double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int k = t;
  for (; k + 7 * NT < n; k += 8 * NT) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += src[k + j * NT];
  }
  for (; k < n; k += NT) acc[0] += src[k];
  red[t] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  for (int h = NT / 2; h > 0; h >>= 1) {
    if (t < h) red[t] += red[t + h];
    __syncthreads();
  }
  return red[0];
}

}  // namespace
}  // namespace trex
