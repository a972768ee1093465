// libtrexhip.so -- Sankoff DP kernels for MI355X (gfx950, CDNA4).
//
// Reference semantics: maraxen/trex src/trex/sankoff.py (run_dp :24-94,
// vectorized_dp :97, run_sankoff :114-188, backtrack_sankoff_jit :191-267).
// Design: one 64-lane wave per workgroup owns SPT*64 consecutive
// sites of ONE tree, so every branch on the topology is wave-uniform and the
// per-tree program (plan.cpp) is read with scalar loads.  Live internal DP
// vectors / cotangents sit in a per-lane LDS stack (Sethi-Ullman slots);
// the DP table is streamed to HBM with sites innermost (16/8-byte stores).
// The cost matrix (and exp(-(C-cmin)/tau)) live in SGPRs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "sankoff_dev.h"
#include "trex_common.h"

namespace trex {

namespace {

thread_local char g_err[512] = "no error";


// --------------------------------------------------------------------------
// per-lane vector helpers (SPT consecutive sites per lane)
// --------------------------------------------------------------------------
template <int SPT>
__device__ __forceinline__ void ld(const float* __restrict__ p, float (&o)[SPT]) {
  if constexpr (SPT == 4) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else if constexpr (SPT == 2) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    o[0] = v.x; o[1] = v.y;
  } else {
    o[0] = *p;
  }
}

template <int SPT>
__device__ __forceinline__ void st(float* __restrict__ p, const float (&o)[SPT]) {
  if constexpr (SPT == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  } else if constexpr (SPT == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(o[0], o[1]);
  } else {
    *p = o[0];
  }
}

template <int SPT>
__device__ __forceinline__ void ld_codes(const int8_t* __restrict__ p, int (&c)[SPT]) {
  if constexpr (SPT == 4) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int s = 0; s < 4; ++s) c[s] = (int)(int8_t)(w >> (8 * s));
  } else if constexpr (SPT == 2) {
    const uint16_t w = *reinterpret_cast<const uint16_t*>(p);
    c[0] = (int)(int8_t)(w & 0xFF);
    c[1] = (int)(int8_t)(w >> 8);
  } else {
    c[0] = *p;
  }
}

template <int SPT>
__device__ __forceinline__ void st_codes(int8_t* __restrict__ p, const int (&c)[SPT]) {
  if constexpr (SPT == 4) {
    uint32_t w = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) w |= (uint32_t)(uint8_t)c[s] << (8 * s);
    *reinterpret_cast<uint32_t*>(p) = w;
  } else if constexpr (SPT == 2) {
    *reinterpret_cast<uint16_t*>(p) = (uint16_t)((uint8_t)c[0] | ((uint8_t)c[1] << 8));
  } else {
    *p = (int8_t)c[0];
  }
}

// --------------------------------------------------------------------------
// cost matrix in SGPRs.  MODE: kHard (min-plus), kSoftK (factored softmin,
// K[i][j] = exp(-(C[i][j]-cmin)/tau) in SGPRs), kSoftDirect (per-row
// stabilised softmin, used when range(C)/tau > 40 would underflow K).
// --------------------------------------------------------------------------

template <int Q>
struct Coef {
  float c[Q][Q];
  float k[Q][Q];
  float cmin;
};


template <int Q>
__device__ __forceinline__ void cost_range(const float* __restrict__ cost_, float& cmin,
                                           float& cmax) {
  const cptr<float> cost = as_const(cost_);
  cmin = INFINITY;
  cmax = -INFINITY;
#pragma unroll
  for (int q = 0; q < Q * Q; ++q) {
    const float v = cost[q];
    cmin = fminf(cmin, v);
    cmax = fmaxf(cmax, v);
  }
  cmin = uniform(cmin);
  cmax = uniform(cmax);
}

// C == C^T (then K == K^T), wave-uniform
template <int Q>
__device__ __forceinline__ bool cost_symmetric(const float* __restrict__ cost_) {
  const cptr<float> cost = as_const(cost_);
  bool sym = true;
#pragma unroll
  for (int i = 0; i < Q; ++i)
#pragma unroll
    for (int j = i + 1; j < Q; ++j) sym = sym && cost[i * Q + j] == cost[j * Q + i];
  return sym;
}

template <int Q, int MODE>
__device__ __forceinline__ void load_coef(const float* __restrict__ cost_, float a, Coef<Q>& cf) {
  float cmax;
  cost_range<Q>(cost_, cf.cmin, cmax);
  const cptr<float> cost = as_const(cost_);
#pragma unroll
  for (int i = 0; i < Q; ++i)
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const float v = cost[i * Q + j];
      cf.c[i][j] = v;
      if constexpr (MODE == kSoftK) cf.k[i][j] = uniform(fast_exp2((cf.cmin - v) * a));
    }
}

// --------------------------------------------------------------------------
// child value D_c (leaf row / LDS slot / dp row / 1e5 sentinel row)
// --------------------------------------------------------------------------
template <int Q, int SPT>
__device__ __forceinline__ void leaf_rows(const int8_t* __restrict__ p, float (&d)[Q][SPT]) {
  int code[SPT];
  ld_codes<SPT>(p, code);
#pragma unroll
  for (int j = 0; j < Q; ++j)
#pragma unroll
    for (int s = 0; s < SPT; ++s) d[j][s] = (code[s] == j) ? 0.0f : kSentinel;
}

template <int Q, int SPT>
__device__ __forceinline__ void fill_sentinel(float (&d)[Q][SPT]) {
#pragma unroll
  for (int j = 0; j < Q; ++j)
#pragma unroll
    for (int s = 0; s < SPT; ++s) d[j][s] = kSentinel;
}

// LDS slot stack: [slot][lane][Q][SPT] -- each lane's vector is contiguous,
// so a slot access is Q*SPT/4 ds_read_b128 / ds_write_b128.
template <int N>
__device__ __forceinline__ void lds_vec_get(const float* p, float (&o)[N]) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int t = 0; t < N / 4; ++t) {
      const float4 v = reinterpret_cast<const float4*>(p)[t];
      o[4 * t] = v.x; o[4 * t + 1] = v.y; o[4 * t + 2] = v.z; o[4 * t + 3] = v.w;
    }
  } else if constexpr (N % 2 == 0) {
#pragma unroll
    for (int t = 0; t < N / 2; ++t) {
      const float2 v = reinterpret_cast<const float2*>(p)[t];
      o[2 * t] = v.x; o[2 * t + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int t = 0; t < N; ++t) o[t] = p[t];
  }
}

template <int N>
__device__ __forceinline__ void lds_vec_put(float* p, const float (&o)[N]) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int t = 0; t < N / 4; ++t)
      reinterpret_cast<float4*>(p)[t] = make_float4(o[4 * t], o[4 * t + 1], o[4 * t + 2], o[4 * t + 3]);
  } else if constexpr (N % 2 == 0) {
#pragma unroll
    for (int t = 0; t < N / 2; ++t) reinterpret_cast<float2*>(p)[t] = make_float2(o[2 * t], o[2 * t + 1]);
  } else {
#pragma unroll
    for (int t = 0; t < N; ++t) p[t] = o[t];
  }
}

template <int Q, int SPT>
__device__ __forceinline__ void lds_get(const float* lds, int slot, int lane, float (&d)[Q][SPT]) {
  float buf[Q * SPT];
  lds_vec_get<Q * SPT>(lds + (slot * kWave + lane) * (Q * SPT), buf);
#pragma unroll
  for (int j = 0; j < Q; ++j)
#pragma unroll
    for (int s = 0; s < SPT; ++s) d[j][s] = buf[j * SPT + s];
}

template <int Q, int SPT>
__device__ __forceinline__ void lds_put(float* lds, int slot, int lane, const float (&d)[Q][SPT]) {
  float buf[Q * SPT];
#pragma unroll
  for (int j = 0; j < Q; ++j)
#pragma unroll
    for (int s = 0; s < SPT; ++s) buf[j * SPT + s] = d[j][s];
  lds_vec_put<Q * SPT>(lds + (slot * kWave + lane) * (Q * SPT), buf);
}

// C[i][code] from SGPR operands (code in [0, Q)); bit-tree select on SSA values
template <int Q>
__device__ __forceinline__ float pick(const float (&row)[Q], int code) {
  float r[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = row[j < Q ? j : 0];
  const bool b0 = (code & 1) != 0;
  const float lo = b0 ? r[1] : r[0];
  if constexpr (Q == 2) return lo;
  if constexpr (Q == 3) return (code & 2) ? r[2] : lo;
  const float hi = b0 ? r[3] : r[2];
  return (code & 2) ? hi : lo;
}


template <int SPT>
__device__ __forceinline__ void bst(rsrc_t r, int voff, int soff, const float (&o)[SPT]) {
  if constexpr (SPT == 2) {
    u32x2 w = {__float_as_uint(o[0]), __float_as_uint(o[1])};
    __builtin_amdgcn_raw_buffer_store_b64(w, r, voff, soff, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o[0]), r, voff, soff, 0);
  }
}

template <int SPT>
__device__ __forceinline__ void bld(rsrc_t r, int voff, int soff, float (&o)[SPT]) {
  if constexpr (SPT == 2) {
    const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    o[0] = __uint_as_float(w.x);
    o[1] = __uint_as_float(w.y);
  } else {
    o[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  }
}

// Site-major DP rows ([row][L][Q]): a lane's SPT consecutive sites x Q states
// are Q*SPT contiguous floats -> one dwordx4 (Q = 4), dwordx3 or dwordx2
// access per site.  voff = site*Q*4 (per lane), soff = row*L*Q*4.
#ifndef TREX_AUX_FWD
#define TREX_AUX_FWD 2
#endif
#ifndef TREX_AUX_FUSED
#define TREX_AUX_FUSED 0
#endif
#ifndef TREX_AUX_ADJ
#define TREX_AUX_ADJ 2
#endif
#ifndef TREX_AUX_MARG
#define TREX_AUX_MARG 2
#endif
// cache policy of the Q <= 4 kernel's DP-row accesses (2 = nt): the
// forward-only kernel's row stores and the adjoint-only kernel's row reads
// and marginal stores stream (C4 forward 620 -> 560 us, adjoint 588 -> ~577
// us); the fused kernel re-reads its rows within the same wave's life, from
// L2 / MALL in part, so its accesses stay temporal
#ifndef TREX_AUX_LEAF
#define TREX_AUX_LEAF 0  // the leaf-tile prefetch loads
#endif
#ifndef TREX_CHERRY_NT
#define TREX_CHERRY_NT 2
#endif
constexpr int kAuxFwdRow = TREX_AUX_FWD, kAuxFusedRow = TREX_AUX_FUSED;
#ifndef TREX_AUX_FUSED_LOAD
#define TREX_AUX_FUSED_LOAD 2
#endif
// the fused kernel's adjoint re-reads of its own rows: nt (each row is read
// once, then dead; with the never-re-read cherry rows also streamed, fused
// 929-934 -> 903-911 us same box, PERFLOG; the stores stay temporal)
constexpr int kAuxFusedLoad = TREX_AUX_FUSED_LOAD;
// the fused kernel's stores of deferred-cherry rows (never re-read)
constexpr int kAuxCherryRow = TREX_CHERRY_NT ? TREX_CHERRY_NT : TREX_AUX_FUSED;
constexpr int kAuxAdjRow = TREX_AUX_ADJ, kAuxMarg = TREX_AUX_MARG;

// AUX: the buffer instruction's cache-policy bits (2 = nt: a streaming
// access that should not displace reused lines)
template <int Q, int SPT, int AUX = 0>
__device__ __forceinline__ void bst_row(rsrc_t r, int voff, int soff, const float (&d)[Q][SPT]) {
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const int vo = voff + s * Q * 4;
    if constexpr (Q == 4) {
      u32x4 w = {__float_as_uint(d[0][s]), __float_as_uint(d[1][s]), __float_as_uint(d[2][s]),
                 __float_as_uint(d[3][s])};
      __builtin_amdgcn_raw_buffer_store_b128(w, r, vo, soff, AUX);
    } else if constexpr (Q == 3) {
      u32x3 w = {__float_as_uint(d[0][s]), __float_as_uint(d[1][s]), __float_as_uint(d[2][s])};
      __builtin_amdgcn_raw_buffer_store_b96(w, r, vo, soff, AUX);
    } else {
      u32x2 w = {__float_as_uint(d[0][s]), __float_as_uint(d[1][s])};
      __builtin_amdgcn_raw_buffer_store_b64(w, r, vo, soff, AUX);
    }
  }
}

template <int Q, int SPT, int AUX = 0>
__device__ __forceinline__ void bld_row(rsrc_t r, int voff, int soff, float (&d)[Q][SPT]) {
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const int vo = voff + s * Q * 4;
    if constexpr (Q == 4) {
      const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(r, vo, soff, AUX);
      d[0][s] = __uint_as_float(w.x); d[1][s] = __uint_as_float(w.y);
      d[2][s] = __uint_as_float(w.z); d[3][s] = __uint_as_float(w.w);
    } else if constexpr (Q == 3) {
      const u32x3 w = __builtin_amdgcn_raw_buffer_load_b96(r, vo, soff, AUX);
      d[0][s] = __uint_as_float(w.x); d[1][s] = __uint_as_float(w.y); d[2][s] = __uint_as_float(w.z);
    } else {
      const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(r, vo, soff, AUX);
      d[0][s] = __uint_as_float(w.x); d[1][s] = __uint_as_float(w.y);
    }
  }
}

#ifdef TREX_DIAG_PAD
// sensitivity probe (diagnostic builds only, wrong timing on purpose, same
// results): TREX_DIAG_SALU / TREX_DIAG_VALU independent dummy scalar /
// vector adds per tree step, to see which issue stream the time follows
__device__ __forceinline__ void diag_pad(float& v) {
  int sd = 0;
#pragma unroll
  for (int i = 0; i < TREX_DIAG_SALU; ++i) asm volatile("s_add_u32 %0, %0, 1" : "+s"(sd));
  float t = 0.0f;
#pragma unroll
  for (int i = 0; i < TREX_DIAG_VALU; ++i) asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(t));
  asm volatile("" ::"s"(sd), "v"(t));
  (void)v;
}
#endif

// s_i = sum_j K_ij u_j for every parent state i.  SYM (K = K^T, symmetric
// C): s_i = sum_j K_ji u_j, accumulated over j with the row pairs (K_j,2p,
// K_j,2p+1) already in SGPRs -- Q / 2 v_pk_fma_f32 per j (8 at Q = 4) instead
// of a pair-wise dot per i (12)
template <int Q, bool SYM>
__device__ __forceinline__ void kvec(const Coef<Q>& cf, const float (&u)[Q], float (&sv)[Q]) {
  if constexpr (SYM && Q % 2 == 0) {
    f2 acc[Q / 2];
#pragma unroll
    for (int p = 0; p < Q / 2; ++p) acc[p] = pk(cf.k[0][2 * p], cf.k[0][2 * p + 1]) * pk(u[0], u[0]);
#pragma unroll
    for (int j = 1; j < Q; ++j)
#pragma unroll
      for (int p = 0; p < Q / 2; ++p)
        acc[p] = __builtin_elementwise_fma(pk(cf.k[j][2 * p], cf.k[j][2 * p + 1]), pk(u[j], u[j]), acc[p]);
#pragma unroll
    for (int p = 0; p < Q / 2; ++p) {
      sv[2 * p] = acc[p].x;
      sv[2 * p + 1] = acc[p].y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < Q; ++i) sv[i] = kdot<Q>(cf.k[i], u);
  }
}

// --------------------------------------------------------------------------
// message M_c[i] = min_j / smin_j (C[i][j] + D_c[j])      (sankoff.py:67-68)
// --------------------------------------------------------------------------
template <int Q, int SPT, int MODE, bool SYM = false>
__device__ __forceinline__ void message(const Coef<Q>& cf, float a, float bcoef,
                                        const float (&d)[Q][SPT], float (&m)[Q][SPT]) {
  if constexpr (MODE == kHard) {
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int s = 0; s < SPT; ++s) {
        float v = cf.c[i][0] + d[0][s];
#pragma unroll
        for (int j = 1; j < Q; ++j) v = fminf(v, cf.c[i][j] + d[j][s]);
        m[i][s] = v;
      }
  } else if constexpr (MODE == kSoftK) {
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      float md = d[0][s];
#pragma unroll
      for (int j = 1; j < Q; ++j) md = fminf(md, d[j][s]);
      const float mda = md * a;
      float u[Q];
#pragma unroll
      for (int j = 0; j < Q; ++j) u[j] = fast_exp2(fmaf(-d[j][s], a, mda));
      const float base = md + cf.cmin;
      float sv[Q];
      kvec<Q, SYM>(cf, u, sv);
#pragma unroll
      for (int i = 0; i < Q; ++i) m[i][s] = fmaf(-bcoef, fast_log2(sv[i]), base);
    }
  } else {
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int s = 0; s < SPT; ++s) {
        float x[Q];
        float mn = INFINITY;
#pragma unroll
        for (int j = 0; j < Q; ++j) {
          x[j] = cf.c[i][j] + d[j][s];
          mn = fminf(mn, x[j]);
        }
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < Q; ++j) acc += fast_exp2((mn - x[j]) * a);
        m[i][s] = fmaf(-bcoef, fast_log2(acc), mn);
      }
  }
}

// --------------------------------------------------------------------------
// adjoint of one child message: acc[i][j] += gbar[i] w[i][j];
// gc[j] = sum_i gbar[i] w[i][j]   (w = tie-averaged argmin or softmax weights)
// In the factored softmin acc holds sum r_i u_j; the K[i][j] factor is
// applied once in the final reduction.
// --------------------------------------------------------------------------
template <int Q, int SPT, int MODE, bool SYM = false>
__device__ __forceinline__ void message_adjoint(const Coef<Q>& cf, float a,
                                                const float (&d)[Q][SPT],
                                                const float (&g)[Q][SPT],
                                                float (&acc)[Q][Q], float (&gc)[Q][SPT]) {
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    if constexpr (MODE == kHard) {
#pragma unroll
      for (int j = 0; j < Q; ++j) gc[j][s] = 0.0f;
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        float x[Q];
        float mn = cf.c[i][0] + d[0][s];
        x[0] = mn;
#pragma unroll
        for (int j = 1; j < Q; ++j) {
          x[j] = cf.c[i][j] + d[j][s];
          mn = fminf(mn, x[j]);
        }
        float cnt = 0.0f;
#pragma unroll
        for (int j = 0; j < Q; ++j) cnt += (x[j] == mn) ? 1.0f : 0.0f;
        const float r = g[i][s] / cnt;
#pragma unroll
        for (int j = 0; j < Q; ++j) {
          const float w = (x[j] == mn) ? r : 0.0f;
          acc[i][j] += w;
          gc[j][s] += w;
        }
      }
    } else if constexpr (MODE == kSoftK) {
      float md = d[0][s];
#pragma unroll
      for (int j = 1; j < Q; ++j) md = fminf(md, d[j][s]);
      const float mda = md * a;
      float u[Q];
#pragma unroll
      for (int j = 0; j < Q; ++j) u[j] = fast_exp2(fmaf(-d[j][s], a, mda));
      float r[Q];
      float sv[Q];
      kvec<Q, SYM>(cf, u, sv);
#pragma unroll
      for (int i = 0; i < Q; ++i) r[i] = g[i][s] * __builtin_amdgcn_rcpf(sv[i]);
#pragma unroll
      for (int i = 0; i < Q; ++i) axpy<Q>(acc[i], r[i], u);
      // t[j] = sum_i r_i K[i][j] (row pairs of K), gc = u * t
      float t[Q];
#pragma unroll
      for (int j = 0; j < Q; ++j) t[j] = r[0] * cf.k[0][j];
#pragma unroll
      for (int i = 1; i < Q; ++i) axpy<Q>(t, r[i], cf.k[i]);
#pragma unroll
      for (int j = 0; j < Q; ++j) gc[j][s] = u[j] * t[j];
    } else {
#pragma unroll
      for (int j = 0; j < Q; ++j) gc[j][s] = 0.0f;
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        float x[Q];
        float mn = INFINITY;
#pragma unroll
        for (int j = 0; j < Q; ++j) {
          x[j] = cf.c[i][j] + d[j][s];
          mn = fminf(mn, x[j]);
        }
        float e[Q];
        float sm = 0.0f;
#pragma unroll
        for (int j = 0; j < Q; ++j) {
          e[j] = fast_exp2((mn - x[j]) * a);
          sm += e[j];
        }
        const float r = g[i][s] * __builtin_amdgcn_rcpf(sm);
#pragma unroll
        for (int j = 0; j < Q; ++j) {
          const float w = r * e[j];
          acc[i][j] += w;
          gc[j][s] += w;
        }
      }
    }
  }
}

// root: score and cotangent of the per-site score      (sankoff.py:187)
template <int Q, int SPT, bool SOFT>
__device__ __forceinline__ void root_score(const float (&d)[Q][SPT], float a, float bcoef,
                                           bool hard_root, float (&score)[SPT],
                                           float (&w)[Q][SPT]) {
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    float mn = d[0][s];
#pragma unroll
    for (int i = 1; i < Q; ++i) mn = fminf(mn, d[i][s]);
    if (!SOFT || hard_root) {
      float cnt = 0.0f;
#pragma unroll
      for (int i = 0; i < Q; ++i) cnt += (d[i][s] == mn) ? 1.0f : 0.0f;
      const float r = 1.0f / cnt;
#pragma unroll
      for (int i = 0; i < Q; ++i) w[i][s] = (d[i][s] == mn) ? r : 0.0f;
      score[s] = mn;
    } else {
      float sm = 0.0f;
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        w[i][s] = fast_exp2((mn - d[i][s]) * a);
        sm += w[i][s];
      }
      const float r = __builtin_amdgcn_rcpf(sm);
#pragma unroll
      for (int i = 0; i < Q; ++i) w[i][s] *= r;
      score[s] = fmaf(-bcoef, fast_log2(sm), mn);
    }
  }
}


// --------------------------------------------------------------------------
// Unified Sankoff kernel: PHASE 1 = forward, 2 = adjoint, 3 = both (fused).
//
// One wave per workgroup = 64*SPT consecutive sites of one tree.  LDS holds
//   [slots][Q][64][SPT] f32  live D vectors (forward) / cotangents (adjoint)
//   [nl][64][SPT]       i8   the tile's leaf states (prologue prefetch)
// Leaf and sentinel children are lookups in per-code tables (message and
// adjoint weights; exact closed forms C[i][code] / one-hot when the 1e5
// sentinel dominates), i.e. no transcendental for half of all children.
// --------------------------------------------------------------------------
struct KArgs {
  const int4* steps;
  const int8_t* leaves;
  const float* cost;
  int n_int, nl, L, tiles, B, n_slots;
  float a, bcoef;
  int hard_root;
  float* dp;            // [B][n_int][L][Q] site-major (fwd writes / adjoint reads)
  float* site_score;    // [B][L] or null
  float* tree_score;    // [B]
  const float* dts;     // [B] or null
  float* marg;          // [B][n_int][L][Q] or null
  int8_t* anc;          // [B][n_int][L] or null
  float* d_cost;        // [Q][Q]
  double* part_tree;    // [B*tiles] per-item score partials
  double* part_dc;      // [Q*Q][B*tiles] per-item dC partials
  int nblocks;          // B * tiles work items (ragged: sum of per-tree tiles)
  // ragged batches (null for uniform batches): per-tree records and the
  // work-item -> tree table of the ragged plan (trex_ragged_plan_build)
  const int* rmeta;     // [B][kRaggedMeta]
  const int* ritem;     // [nblocks] tree of each work item
};

// ragged plan per-tree record (ints): steps offset (in steps), n_int, n_leaves,
// L, first site (site_score offset), first work item, leaf byte offset (lo, hi),
// row-site offset of the tree's DP rows (lo, hi; x Q floats), 2 spare


// LDS map (floats): [0, 128) leaf tables, one row per leaf code (code Q =
// missing leaf / all-1e5 sentinel row): T[code][i] = the child's message at
// 0, W[code][i][j] = its adjoint weight (divided by K_ij in the factored
// form) at kWTab -- both depend on the code only, so every leaf / sentinel
// child is a table lookup in both sweeps; then the slot stack
// [max(n_slots, 1)][64][Q*SPT], then the leaf tile [nl][64*SPT] i8 (raw
// codes, normalised to [0, Q] at use).  The root's cotangent goes to slot 0:
// it is written after the forward has consumed every slot and read by the
// first reverse step (always the root's), before any child cotangent is
// written, and slots are lane-private (a dedicated root slot cost 1 KiB per
// wave: 24 -> 29 waves per CU at C4's 3 slots).
constexpr int kTabFloats = 128;
constexpr int kWTab = 32;  // (Q + 1) Q <= 20 message floats precede the weights
#ifndef TREX_ADJ_RING
#define TREX_ADJ_RING 3
#endif
#ifndef TREX_ADJ_WPE
#define TREX_ADJ_WPE 5
#endif
#ifndef TREX_FUSED_WPE
#define TREX_FUSED_WPE TREX_ADJ_WPE
#endif
#ifndef TREX_FUSED_WPE_MAX
#define TREX_FUSED_WPE_MAX 8
#endif
#ifndef TREX_FWD_WPE
#define TREX_FWD_WPE 6
#endif
constexpr int kAdjRing = TREX_ADJ_RING;  // adjoint DP-row prefetch depth (steps)
constexpr int kPrefetchRows = 64;  // leaf tiles of <= 64 leaves are prefetched

// Persistent waves: the grid holds as many waves as are co-resident; block
// (x = blockIdx % 8, j = blockIdx / 8) walks the items of XCD x's contiguous
// range with stride gridDim/8, so the waves of one XCD always work on
// adjacent tiles (shared L2 lines).  Each item is one (tree, 64*SPT-site
// tile); the next item's leaf tile is loaded into registers while the
// current one computes.
// (An LDS-resident fused variant -- every internal D vector of the tree kept
// in LDS, no adjoint re-read, one wave per SIMD -- measured 2.3x slower on the
// C4 shard and on par for C2; removed in round 3 with the other A/B-only
// variants)
template <int Q, int SPT, int MODE, int PHASE, bool RAGGED, bool SYM = false>
__device__ __forceinline__ void sankoff_body(const KArgs& A, float* lds) {
  static_assert(!RAGGED || SPT == 1, "ragged batches use the SPT=1 kernels");
  constexpr bool SOFT = MODE != kHard;
  constexpr bool FWD = (PHASE & 1) != 0;
  constexpr bool BWD = (PHASE & 2) != 0;
  const int lane = threadIdx.x;
  const int L = A.L;
  const float a = A.a, bcoef = A.bcoef;
  const int nb = A.nblocks;
  const int per = (nb + 7) / 8;
  const int xcd = blockIdx.x & 7;
  const int stride = gridDim.x >> 3;
  const int item_end = min(nb, (xcd + 1) * per);
  int item = xcd * per + (blockIdx.x >> 3);
  if (item >= item_end) return;

  Coef<Q> cf;
  load_coef<Q, MODE>(A.cost, a, cf);

  float* tab = lds;
  float* slots = lds + kTabFloats;
  constexpr int kRootSlot = 0;
  int8_t* lleaf = reinterpret_cast<int8_t*>(slots + (size_t)max(A.n_slots, 1) * Q * kWave * SPT);

  // ---- once per wave: the leaf tables.  Lane c <= Q builds row c from the
  // child row D = (0 at c, 1e5 elsewhere; all 1e5 for c = Q).  When the 1e5
  // sentinel dominates (hard: range(C) < 1e5; soft: exp(-(1e5 - range)/tau)
  // < 2^-64) a present leaf's message is exactly C[i][c] and its weights are
  // one-hot at j = c (x 1/K_ic in the factored form); otherwise (and for the
  // all-1e5 row) the tables hold the general message / weights of that row,
  // i.e. what the per-site code computes for it ----
  {
    float cmn, cmx;
    cost_range<Q>(A.cost, cmn, cmx);
    const float range = cmx - cmn;
    const bool lfast = (MODE != kHard) ? ((kSentinel - range) * a >= 64.0f) : (range < 99000.0f);
    if (lane <= Q) {
      const cptr<float> cost = as_const(A.cost);
      float d1[Q][1], m1[Q][1], g1[Q][1], w1[Q][Q], gc1[Q][1];
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        d1[j][0] = j == lane ? 0.0f : kSentinel;
        g1[j][0] = 1.0f;
      }
#pragma unroll
      for (int i = 0; i < Q; ++i)
#pragma unroll
        for (int j = 0; j < Q; ++j) w1[i][j] = 0.0f;
      if (lfast && lane < Q) {
#pragma unroll
        for (int i = 0; i < Q; ++i) {
          const float cv = cost[i * Q + lane];
          m1[i][0] = cv;
          const float ik = MODE == kSoftK ? fast_exp2((cv - cf.cmin) * a) : 1.0f;
#pragma unroll
          for (int j = 0; j < Q; ++j) w1[i][j] = j == lane ? ik : 0.0f;
        }
      } else {
        message<Q, 1, MODE>(cf, a, bcoef, d1, m1);
        message_adjoint<Q, 1, MODE>(cf, a, d1, g1, w1, gc1);
      }
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        tab[lane * Q + i] = m1[i][0];
#pragma unroll
        for (int j = 0; j < Q; ++j) tab[kWTab + (lane * Q + i) * Q + j] = w1[i][j];
      }
    }
  }

  // leaf-tile prefetch: lane l loads dword (l & 15) of rows 4r + (l >> 4),
  // i.e. 16 loads cover 64 leaf rows of a 64-site tile (4-byte aligned rows)
  // (all 16 loads in flight together: one HBM round trip per tile, where the
  // byte-per-lane path waits once per batch of 8 rows).  Only the forward
  // kernel loops over items and so prefetches the NEXT tile: the adjoint's
  // register footprint is too large to keep a second tile in flight
  constexpr bool PERSIST = PHASE == 1;
  const bool pf = !RAGGED && SPT == 1 && (L & 3) == 0 && A.nl <= kPrefetchRows;
  const int pf_voff = (lane >> 4) * L + (lane & 15) * 4;
  uint32_t pre[kPrefetchRows / 4];
  auto issue_prefetch = [&](int it) {
    const int tr = it / A.tiles;
    const int tl = it - tr * A.tiles;
    const rsrc_t rl = make_rsrc(A.leaves + (size_t)tr * A.nl * L, (uint32_t)((size_t)A.nl * L));
#pragma unroll
    for (int r = 0; r < kPrefetchRows / 4; ++r)
      pre[r] = __builtin_amdgcn_raw_buffer_load_b32(rl, pf_voff, 4 * r * L + tl * kWave, TREX_AUX_LEAF);
  };
  auto store_prefetch = [&]() {
    uint32_t* dst = reinterpret_cast<uint32_t*>(lleaf);
#pragma unroll
    for (int r = 0; r < kPrefetchRows / 4; ++r) {
      const int row = 4 * r + (lane >> 4);
      if (row < A.nl) dst[row * 16 + (lane & 15)] = pre[r];
    }
  };
  if (pf) issue_prefetch(item);
  __syncthreads();  // the tables are written by lanes <= Q, read by all

  do {
    // ---- this item's tree: shape and base offsets ----
    int tree, tile, n_int, nl, Lt;
    size_t leaf_base, rows_base, site_base;  // bytes / row-sites / sites
    cptr<int> prog;
    if constexpr (RAGGED) {
      tree = as_const(A.ritem)[item];
      const cptr<int> m = as_const(A.rmeta) + (size_t)tree * kRaggedMeta;
      n_int = m[1];
      nl = m[2];
      Lt = m[3];
      site_base = (size_t)(uint32_t)m[4];
      tile = item - m[5];
      leaf_base = (size_t)(uint32_t)m[6] | ((size_t)(uint32_t)m[7] << 32);
      rows_base = (size_t)(uint32_t)m[8] | ((size_t)(uint32_t)m[9] << 32);
      prog = as_const(reinterpret_cast<const int*>(A.steps)) + (size_t)m[0] * 4;
    } else {
      tree = item / A.tiles;
      tile = item - tree * A.tiles;
      n_int = A.n_int;
      nl = A.nl;
      Lt = L;
      leaf_base = (size_t)tree * A.nl * L;
      rows_base = (size_t)tree * A.n_int * L;
      site_base = (size_t)tree * L;
      prog = as_const(reinterpret_cast<const int*>(A.steps)) + (size_t)tree * A.n_int * 4;
    }
    const int site = (tile * kWave + lane) * SPT;
    const bool active = site < Lt;
    const int sc = active ? site : 0;

    // ---- leaf tile of this item ----
    if (pf) {
      store_prefetch();
      if (PERSIST && item + stride < item_end) issue_prefetch(item + stride);
    } else {
      const int8_t* lv = A.leaves + leaf_base + sc;
      constexpr int kBatch = 8;
      for (int c0 = 0; c0 < nl; c0 += kBatch) {
        int code[kBatch][SPT];
        const int nb_ = min(kBatch, nl - c0);
#pragma unroll
        for (int u = 0; u < kBatch; ++u)
          if (u < nb_) ld_codes<SPT>(lv + (size_t)(c0 + u) * Lt, code[u]);
#pragma unroll
        for (int u = 0; u < kBatch; ++u)
          if (u < nb_) st_codes<SPT>(lleaf + ((c0 + u) * kWave + lane) * SPT, code[u]);
      }
    }

    const uint32_t treebytes = (uint32_t)((size_t)n_int * Q * Lt * 4);
    const rsrc_t rdp = make_rsrc(A.dp + rows_base * Q, treebytes);
    // inactive lanes address past the buffer: stores drop, loads return 0
    const int voff = active ? site * Q * 4 : 0x7FFFFFF0;
    const int rowbytes = Lt * Q * 4;

    auto child_code = [&](int desc, int (&code)[SPT]) {
      ld_codes<SPT>(lleaf + ((desc & 0xFFFF) * kWave + lane) * SPT, code);
#pragma unroll
      for (int s = 0; s < SPT; ++s) code[s] = ((unsigned)code[s] < (unsigned)Q) ? code[s] : Q;
    };

    float dv[Q][SPT];
    if constexpr (FWD) {
      float prev[Q][SPT];  // previous step's D (register bypass, kChildPrev)
      I4 nxt = load_step(prog, 0);
      for (int k = 0; k < n_int; ++k) {
        const I4 stp = nxt;
        if (k + 1 < n_int) nxt = load_step(prog, k + 1);
        // gather both children (LDS reads in flight together)
        float d[2][Q][SPT];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? stp.y : stp.z;
          const int kind = (desc >> 24) & 3;
          if (desc & kChildPrev) {
#pragma unroll
            for (int j = 0; j < Q; ++j)
#pragma unroll
              for (int s = 0; s < SPT; ++s) d[c][j][s] = prev[j][s];
          } else if (kind == kKindInt) {
            lds_get<Q, SPT>(slots, (desc >> 16) & 0xFF, lane, d[c]);
          } else {
            int code[SPT];
            if (kind == kKindLeaf) {
              child_code(desc, code);
            } else {
#pragma unroll
              for (int s = 0; s < SPT; ++s) code[s] = Q;  // all-1e5 row
            }
#pragma unroll
            for (int s = 0; s < SPT; ++s) {
              float r[Q];
              lds_vec_get<Q>(tab + code[s] * Q, r);
#pragma unroll
              for (int i = 0; i < Q; ++i) d[c][i][s] = r[i];  // already the message
            }
          }
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? stp.y : stp.z;
          float m[Q][SPT];
          if (((desc >> 24) & 3) != kKindInt) {
#pragma unroll
            for (int i = 0; i < Q; ++i)
#pragma unroll
              for (int s = 0; s < SPT; ++s) m[i][s] = d[c][i][s];
          } else {
            // the forward keeps the pair-wise dots in every kernel: the DP
            // table is bitwise the same from the fused, forward-only and
            // ragged launches (the symmetric-K form sums in another order)
            message<Q, SPT, MODE, false>(cf, a, bcoef, d[c], m);
          }
#pragma unroll
          for (int i = 0; i < Q; ++i)
#pragma unroll
            for (int s = 0; s < SPT; ++s) dv[i][s] = (c == 0) ? m[i][s] : dv[i][s] + m[i][s];
        }
        const int row = stp.x & 0xFFFF;
        const int oslot = (stp.x >> 16) & 0xFF;
#ifdef TREX_DIAG_PAD
        diag_pad(dv[0][0]);
#endif
#ifdef TREX_DIAG_NOSTORE
        bst_row<Q, SPT, BWD ? kAuxFusedRow : kAuxFwdRow>(rdp, 0x7FFFFFF0, row * rowbytes, dv);
#elif defined(TREX_DIAG_DROP)
        // probe: the first (DROP > 0) or last (DROP < 0) |DROP| steps' stores dropped
        const bool drop = TREX_DIAG_DROP > 0 ? k < TREX_DIAG_DROP : k >= n_int + TREX_DIAG_DROP;
        bst_row<Q, SPT, BWD ? kAuxFusedRow : kAuxFwdRow>(rdp, drop ? 0x7FFFFFF0 : voff,
                                                        row * rowbytes, dv);
#else
        // rows the adjoint never re-reads (deferred cherries) stream past the
        // caches (nt), so the re-read rows keep more of L2 / MALL: the
        // 128-tree shard 134 -> 128 us, the full batch unchanged (its table
        // is ~10x the MALL); TREX_CHERRY_NT=0 builds the uniform policy
        if (BWD && kAuxCherryRow != kAuxFusedRow && (stp.w & kStepDeferredIn))
          bst_row<Q, SPT, kAuxCherryRow>(rdp, voff, row * rowbytes, dv);
        else
          bst_row<Q, SPT, BWD ? kAuxFusedRow : kAuxFwdRow>(rdp, voff, row * rowbytes, dv);
#endif
        if (!(stp.w & kStepToNext) && oslot != 0xFF) {
          lds_put<Q, SPT>(slots, oslot, lane, dv);
        }
#pragma unroll
        for (int i = 0; i < Q; ++i)
#pragma unroll
          for (int s = 0; s < SPT; ++s) prev[i][s] = dv[i][s];
      }
    } else {
      // adjoint only: the root row comes from the table
      bld_row<Q, SPT>(rdp, voff, (n_int - 1) * rowbytes, dv);
    }

    // ---- root: score + cotangent ----
    float score[SPT], groot[Q][SPT];
    root_score<Q, SPT, SOFT>(dv, a, bcoef, A.hard_root != 0, score, groot);
    if constexpr (FWD) {
      double tot = 0.0;
      if (active) {
#pragma unroll
        for (int s = 0; s < SPT; ++s) tot += (double)score[s];
        if (A.site_score) st<SPT>(A.site_score + site_base + site, score);
      }
      tot = wave_sum_lane0(tot);
      if (lane == 0) A.part_tree[item] = tot;
    }

    if constexpr (BWD) {
      // acc: dC accumulators (in the factored form x K[i][j] at the end; leaf
      // one-hot contributions are pre-divided by K via the IK table)
      float acc[Q][Q];
      const float dscale = A.dts ? as_const(A.dts)[tree] : 1.0f;
      const float f = active ? dscale : 0.0f;
#pragma unroll
      for (int i = 0; i < Q; ++i)
#pragma unroll
        for (int s = 0; s < SPT; ++s) groot[i][s] *= f;
#pragma unroll
      for (int i = 0; i < Q; ++i)
#pragma unroll
        for (int j = 0; j < Q; ++j) acc[i][j] = 0.0f;
      const bool want_marg = A.marg != nullptr;
      const rsrc_t rmg = make_rsrc(want_marg ? A.marg + rows_base * Q : A.dp, treebytes);
      int8_t* at = A.anc ? A.anc + rows_base + sc : nullptr;
      lds_put<Q, SPT>(slots, kRootSlot, lane, groot);

      // DP rows of a step's internal children are loaded one step ahead into
      // the other half of a ping-pong buffer (the loop is unrolled by two so
      // the prefetched registers are consumed in place, never copied -- a
      // copy would force a vmcnt(0) wait at the back edge).  The loads are
      // unconditional (non-internal children read past the buffer: no
      // memory traffic, zeros) so every path issues the same number of VMEM
      // ops and the compiler's vmcnt waits stay partial.
      auto prefetch = [&](const I4& s2, float (&nd)[2][Q][SPT]) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? s2.y : s2.z;
          // deferred cherries (kChildDeferred) are recomputed, not re-read
          const bool internal =
              ((desc >> 24) & 3) == kKindInt && !(desc & kChildDeferred);
#ifdef TREX_DIAG_NOLOAD
          const int vo = 0x7FFFFFF0 + 0 * (internal ? voff : 0);
#else
          const int vo = internal ? voff : 0x7FFFFFF0;
#endif
          const int crow = internal ? (desc & 0xFFFF) : 0;
          bld_row<Q, SPT, FWD ? kAuxFusedLoad : kAuxAdjRow>(rdp, vo, crow * rowbytes, nd[c]);
        }
      };
      float gnext[Q][SPT];  // cotangent handed to the next reverse step (bypass)
      auto bstep = [&](const I4& stp, float (&cd)[2][Q][SPT]) {
        if (stp.w & kStepUnreached) return;
        const int row = stp.x & 0xFFFF;
#ifdef TREX_DIAG_PAD
        diag_pad(acc[0][0]);
#endif
        float g[Q][SPT];
        if (stp.w & kStepToNext) {
#pragma unroll
          for (int i = 0; i < Q; ++i)
#pragma unroll
            for (int s = 0; s < SPT; ++s) g[i][s] = gnext[i][s];
        } else {
          lds_get<Q, SPT>(slots, (stp.w & kStepRoot) ? kRootSlot : ((stp.x >> 16) & 0xFF), lane, g);
        }
        auto leaf_codes = [&](int desc, int kind, int (&code)[SPT]) {
          if (kind == kKindLeaf) {
            child_code(desc, code);
          } else {
#pragma unroll
            for (int s = 0; s < SPT; ++s) code[s] = Q;  // all-1e5 row
          }
        };
        if (stp.w & kStepDeferredIn) {
          // g is the parent's cotangent: this cherry's D is the sum of its two
          // leaf messages (the forward's order, so bit-identical), then the
          // parent -> cherry edge adjoint the parent's step skipped
          float dc[Q][SPT];
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int desc = c == 0 ? stp.y : stp.z;
            int code[SPT];
            leaf_codes(desc, (desc >> 24) & 3, code);
#pragma unroll
            for (int s = 0; s < SPT; ++s) {
              float r[Q];
              lds_vec_get<Q>(tab + code[s] * Q, r);
#pragma unroll
              for (int i = 0; i < Q; ++i) dc[i][s] = (c == 0) ? r[i] : dc[i][s] + r[i];
            }
          }
          float gc[Q][SPT];
          message_adjoint<Q, SPT, MODE, SYM>(cf, a, dc, g, acc, gc);
#pragma unroll
          for (int i = 0; i < Q; ++i)
#pragma unroll
            for (int s = 0; s < SPT; ++s) g[i][s] = gc[i][s];
        }
        if (want_marg) {
          bst_row<Q, SPT, kAuxMarg>(rmg, voff, row * rowbytes, g);
        }
        if (at && active) {
          int best[SPT];
#pragma unroll
          for (int s = 0; s < SPT; ++s) {
            float bv = g[0][s];
            int bi = 0;
#pragma unroll
            for (int i = 1; i < Q; ++i)
              if (g[i][s] > bv) { bv = g[i][s]; bi = i; }
            best[s] = bi;
          }
          st_codes<SPT>(at + (size_t)row * Lt, best);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? stp.y : stp.z;
          const int kind = (desc >> 24) & 3;
          if (kind != kKindInt) {
            // leaf / sentinel child: acc_ij += g_i W[code][i][j] (no cotangent)
            int code[SPT];
            leaf_codes(desc, kind, code);
#pragma unroll
            for (int s = 0; s < SPT; ++s) {
              float w[Q * Q];
              lds_vec_get<Q * Q>(tab + kWTab + code[s] * Q * Q, w);
#pragma unroll
              for (int i = 0; i < Q; ++i) {
                float wr[Q];
#pragma unroll
                for (int j = 0; j < Q; ++j) wr[j] = w[i * Q + j];
                axpy<Q>(acc[i], g[i][s], wr);
              }
            }
          } else {
            float gc[Q][SPT];
            if (desc & kChildDeferred) {
              // the child's step runs this edge (kStepDeferredIn)
#pragma unroll
              for (int j = 0; j < Q; ++j)
#pragma unroll
                for (int s = 0; s < SPT; ++s) gc[j][s] = g[j][s];
            } else {
              message_adjoint<Q, SPT, MODE, SYM>(cf, a, cd[c], g, acc, gc);
            }
            if (desc & kChildPrev) {
#pragma unroll
              for (int j = 0; j < Q; ++j)
#pragma unroll
                for (int s = 0; s < SPT; ++s) gnext[j][s] = gc[j][s];
            } else if (kind == kKindInt) {
              const int cslot = (desc >> 16) & 0xFF;
              if (desc & kStepAccumulate) {
                float old[Q][SPT];
                lds_get<Q, SPT>(slots, cslot, lane, old);
#pragma unroll
                for (int j = 0; j < Q; ++j)
#pragma unroll
                  for (int s = 0; s < SPT; ++s) gc[j][s] += old[j][s];
              }
              lds_put<Q, SPT>(slots, cslot, lane, gc);
            }
          }
        }
      };
      {
      // ring of kRing row buffers: step k's rows were issued kRing - 1 steps
      // earlier (more bytes in flight per wave than a ping-pong; the ring is
      // unrolled so every buffer index is static)
      constexpr int kRing = kAdjRing;
      float buf[kRing][2][Q][SPT];
      I4 sd[kRing];
      const I4 none = {0, 0, 0, 0};  // sentinel children only: prefetch reads nothing
#pragma unroll
      for (int r = 0; r < kRing - 1; ++r) {
        sd[r] = n_int - 1 - r >= 0 ? load_step(prog, n_int - 1 - r) : none;
        prefetch(sd[r], buf[r]);
      }
      I4 nd = n_int - kRing >= 0 ? load_step(prog, n_int - kRing) : none;
      for (int k = n_int - 1; k >= 0; k -= kRing) {
#pragma unroll
        for (int r = 0; r < kRing; ++r) {
          // step k - r uses buf[r]; its freed predecessor slot takes the rows
          // of step k - r - (kRing - 1) (descriptor loaded one round ahead)
          const int w = (r + kRing - 1) % kRing;
          const int j = k - r - (kRing - 1);
          sd[w] = nd;
          prefetch(sd[w], buf[w]);
          nd = j - 1 >= 0 ? load_step(prog, j - 1) : none;
          if (k - r < 0) break;
          bstep(sd[r], buf[r]);
        }
      }
      }

      // ---- per-item dC partial (fixed-order reduce kernel sums the items) ----
      if constexpr (Q == 4) {
        double v16[16];
#pragma unroll
        for (int i = 0; i < Q; ++i)
#pragma unroll
          for (int j = 0; j < Q; ++j) {
            v16[i * Q + j] = (double)acc[i][j];
            if constexpr (MODE == kSoftK) v16[i * Q + j] *= (double)cf.k[i][j];
          }
        const double v = wave_reduce_scatter16(v16, lane);
        if ((lane & 3) == 0) A.part_dc[(size_t)(lane >> 2) * nb + item] = v;
      } else {
#pragma unroll
        for (int i = 0; i < Q; ++i)
#pragma unroll
          for (int j = 0; j < Q; ++j) {
            double v = (double)acc[i][j];
            if constexpr (MODE == kSoftK) v = v * (double)cf.k[i][j];
            v = wave_sum_lane0(v);
            if (lane == 0) A.part_dc[(size_t)(i * Q + j) * nb + item] = v;
          }
      }
    }
    item += stride;
  } while (PERSIST && item < item_end);
}

template <int Q, int SPT, bool SOFT, int PHASE, bool RAGGED = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(PHASE == 1 ? TREX_FWD_WPE : PHASE == 2 ? TREX_ADJ_WPE : TREX_FUSED_WPE, PHASE == 3 ? TREX_FUSED_WPE_MAX : 8)))
void sankoff_kernel(KArgs A) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if constexpr (!SOFT) {
    sankoff_body<Q, SPT, kHard, PHASE, RAGGED>(A, lds);
  } else {
    float cmin, cmax;
    cost_range<Q>(A.cost, cmin, cmax);
    if (use_ktrick(cmin, cmax, A.a)) {
#ifndef TREX_NO_KSYM
      // the adjoint-bearing kernels (the forward-only one measured no gain
      // and would carry a third body's scalar registers: 154 -> 245 spilled)
      if ((PHASE & 2) && cost_symmetric<Q>(A.cost))
        sankoff_body<Q, SPT, kSoftK, PHASE, RAGGED, true>(A, lds);
      else
#endif
        sankoff_body<Q, SPT, kSoftK, PHASE, RAGGED>(A, lds);
    } else
      sankoff_body<Q, SPT, kSoftDirect, PHASE, RAGGED>(A, lds);
  }
}

// --------------------------------------------------------------------------
// trex-exact ancestral reconstruction (sankoff.py:166-185, 191-267)
// --------------------------------------------------------------------------
// RAGGED: bt points at the ragged plan's records (rmeta), the item table
// follows them, then the steps and the backtrack entries (see plan.cpp)
template <int Q, int SPT, bool RAGGED = false>
__global__ __launch_bounds__(kWave) void sankoff_backtrack_kernel(
    const int2* __restrict__ bt, const float* __restrict__ cost, const float* __restrict__ dp,
    int n_int, int L, int tiles, int8_t* __restrict__ anc, const int* __restrict__ rmeta = nullptr,
    int B = 0, int items = 0, int steps = 0) {
  int tree, tile;
  size_t rows_base;
  if constexpr (RAGGED) {
    const int item = blockIdx.x;
    tree = as_const(rmeta + (size_t)B * kRaggedMeta)[item];
    const cptr<int> m = as_const(rmeta) + (size_t)tree * kRaggedMeta;
    n_int = m[1];
    L = m[3];
    tile = item - m[5];
    rows_base = (size_t)(uint32_t)m[8] | ((size_t)(uint32_t)m[9] << 32);
    bt = reinterpret_cast<const int2*>(rmeta + (size_t)B * kRaggedMeta + items + (size_t)steps * 4) +
         m[0];
  } else {
    tree = blockIdx.x / tiles;
    tile = blockIdx.x - tree * tiles;
    rows_base = (size_t)tree * n_int * L;
  }
  const int lane = threadIdx.x;
  const int site = (tile * kWave + lane) * SPT;
  if (site >= L) return;
  float c[Q][Q];
#pragma unroll
  for (int i = 0; i < Q; ++i)
#pragma unroll
    for (int j = 0; j < Q; ++j) c[i][j] = as_const(cost)[i * Q + j];
  const cptr<int> prog = as_const(reinterpret_cast<const int*>(bt)) + (RAGGED ? 0 : (size_t)tree * n_int * 2);
  const size_t rowstride = (size_t)Q * L;  // site-major rows [L][Q]
  const float* dpt = dp + rows_base * Q + (size_t)site * Q;
  int8_t* at = anc + rows_base + site;
  for (int k = 0; k < n_int; ++k) {
    const int2 e = make_int2(prog[2 * k], prog[2 * k + 1]);
    const int x = e.x & 0xFFFF;
    const int kind = (e.x >> 16) & 0xF;
    int out[SPT];
    if (kind == kBtUnreached) {
#pragma unroll
      for (int s = 0; s < SPT; ++s) out[s] = 0;
    } else {
      float d[Q][SPT];
      if (kind == kBtSentinel) {
        fill_sentinel<Q, SPT>(d);
      } else {
        const float* pr = dpt + (size_t)x * rowstride;
#pragma unroll
        for (int t = 0; t < SPT; ++t) {
          if constexpr (Q == 4) {
            const float4 v = reinterpret_cast<const float4*>(pr)[t];
            d[0][t] = v.x; d[1][t] = v.y; d[2][t] = v.z; d[3][t] = v.w;
          } else {
#pragma unroll
            for (int j = 0; j < Q; ++j) d[j][t] = pr[t * Q + j];
          }
        }
      }
      if (kind == kBtRoot) {
#pragma unroll
        for (int s = 0; s < SPT; ++s) {
          float bv = d[0][s];
          int bi = 0;
#pragma unroll
          for (int j = 1; j < Q; ++j)
            if (d[j][s] < bv) { bv = d[j][s]; bi = j; }
          out[s] = bi;
        }
      } else {
        int sp[SPT];
        ld_codes<SPT>(at + (size_t)e.y * L, sp);
#pragma unroll
        for (int s = 0; s < SPT; ++s) {
          float row[Q];
#pragma unroll
          for (int j = 0; j < Q; ++j) {
            float v = c[0][j];
#pragma unroll
            for (int i = 1; i < Q; ++i) v = (sp[s] == i) ? c[i][j] : v;
            row[j] = v;
          }
          float bv = row[0] + d[0][s];
          int bi = 0;
#pragma unroll
          for (int j = 1; j < Q; ++j) {
            const float v = row[j] + d[j][s];
            if (v < bv) { bv = v; bi = j; }
          }
          out[s] = bi;
        }
      }
    }
    st_codes<SPT>(at + (size_t)x * L, out);
  }
}

// dp [B][n_int][L][Q] (site-major, every Q) -> trex VmappedDPTable [B][L][n_all][Q]
__global__ __launch_bounds__(256) void to_trex_layout_kernel(const float* __restrict__ dp,
                                                            const int8_t* __restrict__ leaves,
                                                            int B, int L, int n_all, int nl, int Q,
                                                            float* __restrict__ out) {
  const size_t total = (size_t)B * n_all * L;
  const int ni = n_all - nl;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const int l = (int)(t % L);
    const size_t rest = t / L;
    const int node = (int)(rest % n_all);
    const int b = (int)(rest / n_all);
    float* o = out + (((size_t)b * L + l) * n_all + node) * Q;
    if (node < nl) {
      const int code = leaves[((size_t)b * nl + node) * L + l];
      for (int q = 0; q < Q; ++q) o[q] = (code == q) ? 0.0f : kSentinel;
    } else {
      const float* src = dp + (((size_t)b * ni + (node - nl)) * L + l) * Q;
      for (int q = 0; q < Q; ++q) o[q] = src[q];
    }
  }
}

// --------------------------------------------------------------------------
// host launch helpers
// --------------------------------------------------------------------------
struct Shape {
  int B, L, n_all, nl, ni, Q;
};

int check_shape(const char* fn, int B, int L, int n_all, int Q, Shape* sh) {
  if (B <= 0 || L <= 0 || n_all < 3 || n_all > 65535 || Q < 2)
    return set_error(TREX_E_ARG, "%s: bad shape B=%d L=%d n_all=%d Q=%d", fn, B, L, n_all, Q);
  if (Q > kBigMaxQ)
    return set_error(TREX_E_UNSUPPORTED, "%s: Q=%d > %d not supported by this build (int8 leaf "
                     "codes / ancestral states)", fn, Q, kBigMaxQ);
  sh->B = B;
  sh->L = L;
  sh->n_all = n_all;
  sh->nl = (n_all + 1) / 2;
  sh->ni = n_all - sh->nl;
  sh->Q = Q;
  return TREX_OK;
}

int tiles_for(int L, int spt) { return (L + kWave * spt - 1) / (kWave * spt); }

size_t lds_bytes(int n_slots, int nl, int Q, int spt) {
  const size_t b = (size_t)kTabFloats * 4 + (size_t)std::max(n_slots, 1) * Q * kWave * spt * 4 +
                   (size_t)nl * kWave * spt;
  return (b + 15) & ~(size_t)15;
}

constexpr size_t kLdsPerCu = 160 * 1024;

int device_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return cus;
}

int hip_check(const char* fn) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

int64_t counters_bytes(int B) { return ((int64_t)4 * (B + 1) + 255) / 256 * 256; }

void tau_coefs(float tau, float* a, float* bcoef) {
  if (tau > 0.0f) {
    *a = (float)(1.4426950408889634 / (double)tau);
    *bcoef = (float)((double)tau * 0.6931471805599453);
  } else {
    *a = 0.0f;
    *bcoef = 0.0f;
  }
}

// persistent grid: as many single-wave blocks as are co-resident (occupancy
// x CUs), a multiple of 8 (one share per XCD), never more than the items
template <class K>
int persistent_grid(K kernel, size_t lds, int nitems) {
  static std::mutex mu;
  static int cus = 0;
  struct Entry { const void* k; size_t lds; int occ; };
  static Entry cache[64];
  static int ncache = 0;
  int occ = 0;
  {
    std::lock_guard<std::mutex> g(mu);
    if (cus == 0) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    }
    for (int i = 0; i < ncache; ++i)
      if (cache[i].k == (const void*)kernel && cache[i].lds == lds) occ = cache[i].occ;
    if (occ == 0) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, kWave, lds) != hipSuccess ||
          occ <= 0)
        occ = 4;
      if (ncache < 64) cache[ncache++] = Entry{(const void*)kernel, lds, occ};
    }
  }
#ifdef TREX_FWD_OCC_CAP
  occ = std::min(occ, TREX_FWD_OCC_CAP);
#endif
  const long resident = (long)cus * occ / 8 * 8;
  const long want = ((long)nitems + 7) / 8 * 8;
  return (int)std::max(8L, std::min(resident, want));
}

template <int Q, int SPT, bool SOFT>
void launch_phase(int phase, size_t lds, hipStream_t st, const KArgs& A) {
  auto go = [&](auto kernel) {
    const int grid = phase == 1 ? persistent_grid(kernel, lds, A.nblocks) : (A.nblocks + 7) / 8 * 8;
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kWave), lds, st, A);
  };
  if (phase == 1)
    go(sankoff_kernel<Q, SPT, SOFT, 1>);
  else if (phase == 2)
    go(sankoff_kernel<Q, SPT, SOFT, 2>);
  else
    go(sankoff_kernel<Q, SPT, SOFT, 3>);
}

// one site per lane (SPT = 1): two sites per lane doubled the adjoint's
// VGPRs and was slower at every grid measured
template <int Q>
void dispatch_q(int phase, bool soft, size_t lds, hipStream_t st, const KArgs& A) {
  if (soft) launch_phase<Q, 1, true>(phase, lds, st, A);
  else launch_phase<Q, 1, false>(phase, lds, st, A);
}

// common entry: validates, fills KArgs, launches one phase
// Q <= 4 on a small grid (few trees x few sites: C2 is one tree, 157 waves
// of 64 sites for 1 024 SIMDs) runs the state-parallel kernel instead: 4
// lanes per site (one per parent state), 16 sites per wave, 4x the waves and
// a quarter of the per-lane work on the serial node chain.
// TREX_WIDE_SMALLQ=0 / 1 forces the choice (A/B).
bool wide_small_q(int B, int L, int Q) {
  if (Q > 4) return false;
  // read per call (tests run both kernels in one process)
  const char* e = std::getenv("TREX_WIDE_SMALLQ");
  if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1';
  // up to ~1.5 64-site waves per CU on the lane-per-site kernel (measured
  // on 256 CUs, 32-taxa trees x 5 000 sites: 158 waves 43.8 -> 40.4 us, 316
  // waves 46.5 -> 44.9 us, 632 waves 48.2 vs 51.8 us (lane-per-site wins);
  // C2 71 -> 67 us; a C4 shard, 10 000 waves, is 2.2x slower
  // state-parallel).  Scaled by the CU count (a CPX partition has 32 CUs).
  return (int64_t)B * ((L + kWave - 1) / kWave) * 2 <= (int64_t)3 * device_cus();
}

// Grids of at most about one state-parallel wave per SIMD (C2: one tree x
// 625 16-site items) run the staged kernel (sankoff_staged.hip): one
// workgroup of waves per item, the tree's levels spread over the waves, so
// the serial chain is the tree height instead of every internal node.
// TREX_STAGED=0 / 1 forces it off / on (whenever its LDS fits; A/B, tests).
bool use_staged(int B, int L, int Q, int ni, int nl, int phase) {
  if (staged_lds_bytes(ni, nl, Q, phase) > kLdsPerCu) return false;
  const char* e = std::getenv("TREX_STAGED");  // read per call (tests flip it)
  if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1';
  return (int64_t)B * wide_tiles(L, Q) <= (int64_t)4 * device_cus();
}

int run_phase(const char* fn, int phase, const int32_t* plan, int n_slots, const int8_t* leaves,
              const float* cost, int B, int L, int n_all, int Q, float tau, unsigned flags,
              float* dp, float* site_score, float* tree_score, const float* dts, float* d_cost,
              float* marg, int8_t* anc, void* workspace, int64_t workspace_bytes, void* stream);

}  // namespace

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

namespace {

int run_phase(const char* fn, int phase, const int32_t* plan, int n_slots, const int8_t* leaves,
              const float* cost, int B, int L, int n_all, int Q, float tau, unsigned flags,
              float* dp, float* site_score, float* tree_score, const float* dts, float* d_cost,
              float* marg, int8_t* anc, void* workspace, int64_t workspace_bytes, void* stream) {
  Shape s;
  if (int e = check_shape(fn, B, L, n_all, Q, &s)) return e;
  if (!plan || !leaves || !cost || !workspace)
    return set_error(TREX_E_ARG, "%s: null pointer argument", fn);
  if ((phase & 1) && !tree_score) return set_error(TREX_E_ARG, "%s: tree_score is required", fn);
  if ((phase & 2) && (!dp || !d_cost))
    return set_error(TREX_E_ARG, "%s: dp and d_cost are required", fn);
  if (!nonneg_finite_f32(tau))
    return set_error(TREX_E_ARG, "%s: tau must be finite and >= 0 (got %g)", fn, tau);
  // 4 < Q <= 20: the kept s rows of the fused site kernel are optional -- a
  // workspace without them (site_srow_offset bytes) makes it recompute them
  const bool srow_room = workspace_bytes >= trex_workspace_bytes(B, L, n_all, Q);
  const int64_t min_ws = (Q > 4 && Q <= kSiteMaxQ) ? site_srow_offset(B, L, Q)
                                                   : trex_workspace_bytes(B, L, n_all, Q);
  if (workspace_bytes < min_ws) return set_error(TREX_E_ARG, "%s: workspace too small", fn);
  if (n_slots < 0) return set_error(TREX_E_ARG, "%s: bad n_slots", fn);
  if (flags & ~TREX_FLAG_HARD_ROOT) return set_error(TREX_E_ARG, "%s: unknown flags 0x%x", fn, flags);
  // plan info[0]: stack depth | (lane-program slots + 1) << 16
  const int lp_slots = ((n_slots >> 16) & 0xFF) - 1;
  n_slots &= 0xFFFF;
  if (n_slots > 250) return set_error(TREX_E_ARG, "%s: bad n_slots", fn);
  if (Q > 4 || wide_small_q(B, L, Q)) {
    WideCall c;
    c.phase = phase;
    c.soft = tau > 0.0f;
    c.steps = plan + TREX_PLAN_HEADER_INTS;
    c.leaves = leaves;
    c.cost = cost;
    c.B = B;
    c.L = L;
    c.nl = s.nl;
    c.ni = s.ni;
    c.Q = Q;
    c.n_slots = n_slots;
    tau_coefs(tau, &c.a, &c.bcoef);
    c.hard_root = (flags & TREX_FLAG_HARD_ROOT) ? 1 : 0;
    c.dp = dp;
    c.site_score = site_score;
    c.tree_score = tree_score;
    c.dts = dts;
    c.marg = marg;
    c.anc = anc;
    c.d_cost = d_cost;
    c.workspace = workspace;
    c.stream = stream;
    if (Q > kWideMaxQ) return bigq_run(fn, c);  // 64 < Q <= 128 (sankoff_bigq.hip)
    const int32_t* staged = plan + TREX_PLAN_HEADER_INTS + (int64_t)B * s.ni * 6;
    const int32_t* lanes = staged + (int64_t)B * staged_tree_ints(s.ni);
    if (site_eligible(c, lp_slots)) {
      // the lane-per-site kernel (sankoff_site.hip) takes the call when the
      // cost matrix allows the factored softmin -- decided on the device: the
      // state-parallel kernel runs first, gated (every workgroup checks the
      // cost range and exits when the site kernel takes the call; workgroup
      // 0 writes K, K^T and the flag into the workspace tail), then the site
      // kernel (exits unless the flag is set), then one reduce that sums
      // whichever kernel's partials the flag names
      char* tail = static_cast<char*>(workspace) + wide_workspace_bytes(B, L, Q);
      int* flag = reinterpret_cast<int*>(tail - 128);
      float* kg = reinterpret_cast<float*>(tail - 3456);  // K and K^T
      c.site_flag = flag;
      c.site_kg = kg;
      if (phase == 3 && srow_room && site_srow_on())
        c.site_srow = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                               site_srow_offset(B, L, Q));
      if (int e = wide_run(fn, c, /*reduce=*/false)) return e;
      if (int e = site2_on(lp_slots, c.nl, c.ni) ? site2_run(fn, c, lanes, lp_slots, flag, kg)
                                                 : site_run(fn, c, lanes, lp_slots, flag, kg))
        return e;
      return partial_reduce(fn, static_cast<double*>(workspace),
                            static_cast<double*>(workspace) + (int64_t)B * wide_tiles(L, Q), B,
                            wide_tiles(L, Q), Q, phase, tree_score, d_cost, stream, nullptr, 0, 0,
                            1, flag, site_tiles(L));
    }
    if (use_staged(B, L, Q, s.ni, s.nl, phase)) return staged_run(fn, c, staged);
    return wide_run(fn, c);
  }
  if ((int64_t)s.ni * L * Q * 4 > 0x7FFFFFF0LL)
    return set_error(TREX_E_UNSUPPORTED, "%s: one tree's DP table exceeds 2 GiB", fn);
  const int tiles = tiles_for(L, 1);
  const size_t lds = lds_bytes(n_slots, s.nl, Q, 1);
  if (lds > 65536) return set_error(TREX_E_UNSUPPORTED, "%s: LDS stack too deep", fn);
  if ((int64_t)B * tiles > 0x7FFFFFFF) return set_error(TREX_E_ARG, "%s: grid too large", fn);
  KArgs A;
  A.rmeta = nullptr;
  A.ritem = nullptr;
  A.steps = reinterpret_cast<const int4*>(plan + TREX_PLAN_HEADER_INTS);
  A.leaves = leaves;
  A.cost = cost;
  A.n_int = s.ni;
  A.nl = s.nl;
  A.L = L;
  A.tiles = tiles;
  A.B = B;
  A.n_slots = n_slots;
  tau_coefs(tau, &A.a, &A.bcoef);
  A.hard_root = (flags & TREX_FLAG_HARD_ROOT) ? 1 : 0;
  A.dp = dp;
  A.site_score = site_score;
  A.tree_score = tree_score;
  A.dts = dts;
  A.marg = marg;
  A.anc = anc;
  A.d_cost = d_cost;
  // workspace: per-item partials [B*tiles] + [Q*Q][B*tiles] doubles
  char* w = static_cast<char*>(workspace) + counters_bytes(B);
  A.part_tree = reinterpret_cast<double*>(w);
  A.nblocks = B * tiles;
  A.part_dc = A.part_tree + A.nblocks;
  const bool soft = tau > 0.0f;
  hipStream_t st = (hipStream_t)stream;
  switch (Q) {
    case 2: dispatch_q<2>(phase, soft, lds, st, A); break;
    case 3: dispatch_q<3>(phase, soft, lds, st, A); break;
    case 4: dispatch_q<4>(phase, soft, lds, st, A); break;
  }
  if (int e = hip_check(fn)) return e;
  return partial_reduce(fn, A.part_tree, A.part_dc, B, tiles, Q, phase, tree_score, d_cost, stream);
}

template <int Q, bool SOFT>
void launch_ragged(int phase, size_t lds, hipStream_t st, const KArgs& A) {
  auto go = [&](auto kernel) {
    const int grid = phase == 1 ? persistent_grid(kernel, lds, A.nblocks) : (A.nblocks + 7) / 8 * 8;
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kWave), lds, st, A);
  };
  if (phase == 1)
    go(sankoff_kernel<Q, 1, SOFT, 1, true>);
  else if (phase == 2)
    go(sankoff_kernel<Q, 1, SOFT, 2, true>);
  else
    go(sankoff_kernel<Q, 1, SOFT, 3, true>);
}

}  // namespace

}  // namespace trex

using namespace trex;

extern "C" const char* trex_last_error(void) { return g_err; }

extern "C" int trex_version(void) { return 10; }

extern "C" int trex_dp_site_major(int Q) {
  (void)Q;
  return 1;  // every Q since v4 (Q <= 4 used [n_int][Q][L] before)
}

extern "C" int64_t trex_workspace_bytes(int B, int L, int n_all, int Q) {
  if (B <= 0 || L <= 0 || Q <= 0) return 0;
  if (Q > kWideMaxQ) return bigq_workspace_bytes(B, L, Q);
  if (Q > kSiteMaxQ) return wide_workspace_bytes(B, L, Q);
  if (Q > 4) {  // + the fused lane-per-site kernel's s rows
    const int64_t ni = n_all - (n_all + 1) / 2;
    return site_srow_offset(B, L, Q) + (int64_t)B * std::max<int64_t>(ni, 0) * L * Q * 4;
  }
  const int64_t nb = (int64_t)B * tiles_for(L, 1);
  const int64_t narrow = counters_bytes(B) + nb * 8 * (1 + (int64_t)Q * Q) + (int64_t)Q * Q * B * 8 + 256;
  // small grids may run the state-parallel wide kernel (G = 4): room for both
  return std::max<int64_t>(narrow, wide_workspace_bytes(B, L, Q));
}

extern "C" int trex_workspace_init(void* workspace, int64_t workspace_bytes, void* stream) {
  if (!workspace || workspace_bytes <= 0)
    return set_error(TREX_E_ARG, "trex_workspace_init: bad arguments");
  if (hipMemsetAsync(workspace, 0, (size_t)workspace_bytes, (hipStream_t)stream) != hipSuccess)
    return hip_check("trex_workspace_init");
  return hip_check("trex_workspace_init");
}

extern "C" int trex_sankoff_fwd(const int32_t* plan, int n_slots, const int8_t* leaves,
                                const float* cost, int B, int L, int n_all, int Q, float tau,
                                unsigned flags, float* dp, float* site_score, float* tree_score,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  if (!dp)
    return set_error(TREX_E_UNSUPPORTED,
                     "trex_sankoff_fwd: dp is required (the reference returns the table)");
  return run_phase("trex_sankoff_fwd", 1, plan, n_slots, leaves, cost, B, L, n_all, Q, tau, flags,
                   dp, site_score, tree_score, nullptr, nullptr, nullptr, nullptr, workspace,
                   workspace_bytes, stream);
}

extern "C" int trex_sankoff_bwd(const int32_t* plan, int n_slots, const int8_t* leaves,
                                const float* cost, int B, int L, int n_all, int Q, float tau,
                                unsigned flags, const float* dp, const float* d_tree_score,
                                float* d_cost, float* marginals, int8_t* anc_states,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  return run_phase("trex_sankoff_bwd", 2, plan, n_slots, leaves, cost, B, L, n_all, Q, tau, flags,
                   const_cast<float*>(dp), nullptr, nullptr, d_tree_score, d_cost, marginals,
                   anc_states, workspace, workspace_bytes, stream);
}

extern "C" int trex_sankoff_fwd_bwd(const int32_t* plan, int n_slots, const int8_t* leaves,
                                    const float* cost, int B, int L, int n_all, int Q, float tau,
                                    unsigned flags, float* dp, float* site_score,
                                    float* tree_score, const float* d_tree_score, float* d_cost,
                                    float* marginals, int8_t* anc_states, void* workspace,
                                    int64_t workspace_bytes, void* stream) {
  return run_phase("trex_sankoff_fwd_bwd", 3, plan, n_slots, leaves, cost, B, L, n_all, Q, tau,
                   flags, dp, site_score, tree_score, d_tree_score, d_cost, marginals, anc_states,
                   workspace, workspace_bytes, stream);
}

extern "C" int trex_sankoff_backtrack(const int32_t* plan, int backtrack_ok, const float* cost,
                                      const float* dp, int B, int L, int n_all, int Q,
                                      int8_t* anc_states, void* stream) {
  Shape s;
  if (int e = check_shape("trex_sankoff_backtrack", B, L, n_all, Q, &s)) return e;
  if (!backtrack_ok)
    return set_error(TREX_E_TOPOLOGY,
                     "trex_sankoff_backtrack: the reference backtrack does not terminate on this "
                     "topology (cyclic child references)");
  if (!plan || !cost || !dp || !anc_states)
    return set_error(TREX_E_ARG, "trex_sankoff_backtrack: null pointer argument");
  const int32_t* bt32 = plan + TREX_PLAN_HEADER_INTS + (int64_t)B * s.ni * 4;
  if (Q > kWideMaxQ) return bigq_backtrack(bt32, cost, dp, B, L, s.ni, Q, anc_states, stream);
  // every uniform batch: the split-lane kernels of sankoff_wide.hip (4 lanes
  // per site for Q <= 4, 8 for Q <= 32, one lane per site for codons); the
  // sites-per-lane sankoff_backtrack_kernel serves ragged Q <= 4 batches
  return wide_backtrack(bt32, cost, dp, B, L, s.ni, Q, anc_states, stream);
}

extern "C" int trex_dp_to_trex_layout(const float* dp, const int8_t* leaves, int B, int L,
                                      int n_all, int Q, float* out, void* stream) {
  if (B <= 0 || L <= 0 || n_all < 3 || Q < 2 || Q > kBigMaxQ || !dp || !leaves || !out)
    return set_error(TREX_E_ARG, "trex_dp_to_trex_layout: bad arguments");
  const int nl = (n_all + 1) / 2;
  const size_t total = (size_t)B * n_all * L;
  const int grid = (int)std::min<size_t>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(to_trex_layout_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, dp,
                     leaves, B, L, n_all, nl, Q, out);
  return hip_check("trex_dp_to_trex_layout");
}

// ---------------------------------------------------------------------------
// Ragged batches (trees of different n_all / L in one launch; plan from
// trex_ragged_plan_build).  Packed layouts: leaves [sum n_leaves_b * L_b]
// int8 (tree b at its leaf offset, [n_leaves_b][L_b]); dp / marginals
// [sum n_int_b * L_b][Q] f32 (tree b: [n_int_b][L_b][Q]); site_score
// [sum L_b]; anc_states [sum n_int_b * L_b] int8.
// ---------------------------------------------------------------------------
extern "C" int64_t trex_ragged_workspace_bytes(int64_t items, int Q) {
  if (items <= 0 || Q <= 0) return 0;
  if (Q > kWideMaxQ) return items * 8 * (1 + (int64_t)Q * Q) + 256;  // partials per item
  if (Q > 4) return wide_ragged_workspace_bytes(items, Q);  // partials per wave
  return items * 8 * (1 + (int64_t)Q * Q) + 256;
}

extern "C" int trex_sankoff_ragged(int phase, const int32_t* plan, int B, int n_slots, int max_nl,
                                   int64_t items, const int8_t* leaves, const float* cost, int Q,
                                   float tau, unsigned flags, float* dp, float* site_score,
                                   float* tree_score, const float* d_tree_score, float* d_cost,
                                   float* marginals, int8_t* anc_states, void* workspace,
                                   int64_t workspace_bytes, void* stream) {
  const char* fn = "trex_sankoff_ragged";
  if (phase < 1 || phase > 3) return set_error(TREX_E_ARG, "%s: phase must be 1, 2 or 3", fn);
  if (B <= 0 || items <= 0 || items > 0x7FFFFFFF || max_nl < 2 || Q < 2)
    return set_error(TREX_E_ARG, "%s: bad shape B=%d items=%lld max_nl=%d Q=%d", fn, B,
                     (long long)items, max_nl, Q);
  if (Q > kBigMaxQ)
    return set_error(TREX_E_UNSUPPORTED, "%s: Q=%d > %d not supported by this build (int8 leaf "
                     "codes / ancestral states)", fn, Q, kBigMaxQ);
  if (!plan || !leaves || !cost || !workspace || !dp)
    return set_error(TREX_E_ARG, "%s: null pointer argument", fn);
  if ((phase & 1) && !tree_score) return set_error(TREX_E_ARG, "%s: tree_score is required", fn);
  if ((phase & 2) && !d_cost) return set_error(TREX_E_ARG, "%s: d_cost is required", fn);
  if (!nonneg_finite_f32(tau))
    return set_error(TREX_E_ARG, "%s: tau must be finite and >= 0 (got %g)", fn, tau);
  if (workspace_bytes < trex_ragged_workspace_bytes(items, Q))
    return set_error(TREX_E_ARG, "%s: workspace too small", fn);
  if (n_slots < 0 || n_slots > 250) return set_error(TREX_E_ARG, "%s: bad n_slots", fn);
  if (flags & ~TREX_FLAG_HARD_ROOT) return set_error(TREX_E_ARG, "%s: unknown flags 0x%x", fn, flags);
  if (Q > 4) {
    // protein / codon alphabets: the state-parallel kernel, each 64-site
    // item split over ceil(64 / sites-per-wave) waves
    const int* meta = plan + TREX_PLAN_HEADER_INTS;
    WideCall c;
    c.phase = phase;
    c.soft = tau > 0.0f;
    c.steps = meta + (size_t)B * kRaggedMeta + items;
    c.leaves = leaves;
    c.cost = cost;
    c.B = B;
    c.L = 0;
    c.nl = max_nl;
    c.ni = max_nl - 1;
    c.Q = Q;
    c.n_slots = n_slots;
    tau_coefs(tau, &c.a, &c.bcoef);
    c.hard_root = (flags & TREX_FLAG_HARD_ROOT) ? 1 : 0;
    c.dp = dp;
    c.site_score = site_score;
    c.tree_score = tree_score;
    c.dts = d_tree_score;
    c.marg = marginals;
    c.anc = anc_states;
    c.d_cost = d_cost;
    c.workspace = workspace;
    c.stream = stream;
    if (Q > kWideMaxQ) return bigq_ragged_run(fn, c, meta, meta + (size_t)B * kRaggedMeta, items);
    return wide_ragged_run(fn, c, meta, meta + (size_t)B * kRaggedMeta, items);
  }
  const size_t lds = lds_bytes(n_slots, max_nl, Q, 1);
  if (lds > 65536) return set_error(TREX_E_UNSUPPORTED, "%s: LDS stack too deep", fn);
  KArgs A;
  const int* meta = plan + TREX_PLAN_HEADER_INTS;
  A.rmeta = meta;
  A.ritem = meta + (size_t)B * kRaggedMeta;
  A.steps = reinterpret_cast<const int4*>(A.ritem + items);
  A.leaves = leaves;
  A.cost = cost;
  A.n_int = 0;
  A.nl = max_nl;
  A.L = 0;
  A.tiles = 0;
  A.B = B;
  A.n_slots = n_slots;
  tau_coefs(tau, &A.a, &A.bcoef);
  A.hard_root = (flags & TREX_FLAG_HARD_ROOT) ? 1 : 0;
  A.dp = dp;
  A.site_score = site_score;
  A.tree_score = tree_score;
  A.dts = d_tree_score;
  A.marg = marginals;
  A.anc = anc_states;
  A.d_cost = d_cost;
  A.nblocks = (int)items;
  A.part_tree = reinterpret_cast<double*>(workspace);
  A.part_dc = A.part_tree + items;
  const bool soft = tau > 0.0f;
  hipStream_t st = (hipStream_t)stream;
  switch (Q) {
    case 2: soft ? launch_ragged<2, true>(phase, lds, st, A) : launch_ragged<2, false>(phase, lds, st, A); break;
    case 3: soft ? launch_ragged<3, true>(phase, lds, st, A) : launch_ragged<3, false>(phase, lds, st, A); break;
    case 4: soft ? launch_ragged<4, true>(phase, lds, st, A) : launch_ragged<4, false>(phase, lds, st, A); break;
  }
  if (int e = hip_check(fn)) return e;
  return partial_reduce(fn, A.part_tree, A.part_dc, B, 0, Q, phase, tree_score, d_cost, stream,
                        meta + 5, kRaggedMeta, (int)items);
}

extern "C" int trex_sankoff_ragged_backtrack(const int32_t* plan, int B, int64_t items,
                                             int64_t steps, int backtrack_ok, const float* cost,
                                             const float* dp, int Q, int8_t* anc_states,
                                             void* stream) {
  const char* fn = "trex_sankoff_ragged_backtrack";
  if (B <= 0 || items <= 0 || items > 0x7FFFFFFF || steps <= 0 || Q < 2)
    return set_error(TREX_E_ARG, "%s: bad arguments", fn);
  if (Q > kBigMaxQ)
    return set_error(TREX_E_UNSUPPORTED, "%s: Q=%d > %d not supported by this build", fn, Q,
                     kBigMaxQ);
  if (!backtrack_ok)
    return set_error(TREX_E_TOPOLOGY,
                     "%s: the reference backtrack does not terminate on this batch (cyclic child "
                     "references)", fn);
  if (!plan || !cost || !dp || !anc_states) return set_error(TREX_E_ARG, "%s: null pointer", fn);
  const int* meta = plan + TREX_PLAN_HEADER_INTS;
  if (Q > kWideMaxQ) return bigq_ragged_backtrack(meta, B, items, steps, cost, dp, Q, anc_states, stream);
  if (Q > 4) return wide_ragged_backtrack(meta, B, items, steps, cost, dp, Q, anc_states, stream);
  hipStream_t st = (hipStream_t)stream;
#define TREX_RBT(QQ)                                                                          \
  hipLaunchKernelGGL((sankoff_backtrack_kernel<QQ, 1, true>), dim3((int)items), dim3(kWave), 0, \
                     st, nullptr, cost, dp, 0, 0, 0, anc_states, meta, B, (int)items, (int)steps);
  switch (Q) {
    case 2: TREX_RBT(2) break;
    case 3: TREX_RBT(3) break;
    case 4: TREX_RBT(4) break;
  }
#undef TREX_RBT
  return hip_check(fn);
}
