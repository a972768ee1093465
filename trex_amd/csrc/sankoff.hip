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

#include "trex_common.h"

namespace trex {

namespace {

thread_local char g_err[512] = "no error";

constexpr float kSentinel = 1e5f;  // sankoff.py:152
constexpr int kWave = 64;
constexpr int kKindSent = 0, kKindLeaf = 1, kKindInt = 2;

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

__device__ __forceinline__ float uniform(float x) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }

// --------------------------------------------------------------------------
// cost matrix in SGPRs; K[i][j] = exp(-(C[i][j]-cmin)/tau) for the softmin
// --------------------------------------------------------------------------
template <int Q>
struct Coef {
  float c[Q][Q];
  float k[Q][Q];
  float cmin;
  bool ktrick;  // all K >= exp(-40): the factored softmin is exact to fp32
};

template <int Q, bool SOFT>
__device__ __forceinline__ void load_coef(const float* __restrict__ cost, float a, Coef<Q>& cf) {
  float cmin = INFINITY, cmax = -INFINITY;
#pragma unroll
  for (int i = 0; i < Q; ++i)
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const float v = uniform(cost[i * Q + j]);
      cf.c[i][j] = v;
      cmin = fminf(cmin, v);
      cmax = fmaxf(cmax, v);
    }
  cf.cmin = uniform(cmin);
  cf.ktrick = false;
  if constexpr (SOFT) {
    // log2(e^40) = 57.7: range/tau <= 40
    cf.ktrick = (cmax - cmin) * a <= 57.70780f;
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int j = 0; j < Q; ++j) cf.k[i][j] = uniform(fast_exp2((cf.cmin - cf.c[i][j]) * a));
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

template <int Q, int SPT>
__device__ __forceinline__ void lds_get(const float* lds, int slot, int lane, float (&d)[Q][SPT]) {
#pragma unroll
  for (int j = 0; j < Q; ++j) ld<SPT>(lds + ((slot * Q + j) * kWave + lane) * SPT, d[j]);
}

template <int Q, int SPT>
__device__ __forceinline__ void lds_put(float* lds, int slot, int lane, const float (&d)[Q][SPT]) {
#pragma unroll
  for (int j = 0; j < Q; ++j) st<SPT>(lds + ((slot * Q + j) * kWave + lane) * SPT, d[j]);
}

// --------------------------------------------------------------------------
// message M_c[i] = min_j / smin_j (C[i][j] + D_c[j])      (sankoff.py:67-68)
// --------------------------------------------------------------------------
template <int Q, int SPT, bool SOFT>
__device__ __forceinline__ void message(const Coef<Q>& cf, float a, float bcoef,
                                        const float (&d)[Q][SPT], float (&m)[Q][SPT]) {
  if constexpr (!SOFT) {
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int s = 0; s < SPT; ++s) {
        float v = cf.c[i][0] + d[0][s];
#pragma unroll
        for (int j = 1; j < Q; ++j) v = fminf(v, cf.c[i][j] + d[j][s]);
        m[i][s] = v;
      }
  } else {
    if (cf.ktrick) {
#pragma unroll
      for (int s = 0; s < SPT; ++s) {
        float md = d[0][s];
#pragma unroll
        for (int j = 1; j < Q; ++j) md = fminf(md, d[j][s]);
        float u[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) u[j] = fast_exp2((md - d[j][s]) * a);
        const float base = md + cf.cmin;
#pragma unroll
        for (int i = 0; i < Q; ++i) {
          float acc = cf.k[i][0] * u[0];
#pragma unroll
          for (int j = 1; j < Q; ++j) acc = fmaf(cf.k[i][j], u[j], acc);
          m[i][s] = base - bcoef * fast_log2(acc);
        }
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
          m[i][s] = mn - bcoef * fast_log2(acc);
        }
    }
  }
}

// --------------------------------------------------------------------------
// adjoint of one child message: acc[i][j] += gbar[i] w[i][j];
// gc[j] = sum_i gbar[i] w[i][j]   (w = tie-averaged argmin or softmax weights)
// In the factored softmin acc holds sum r_i u_j; the K[i][j] factor is
// applied once in the final reduction.
// --------------------------------------------------------------------------
template <int Q, int SPT, bool SOFT, bool WANT_GC>
__device__ __forceinline__ void message_adjoint(const Coef<Q>& cf, float a,
                                                const float (&d)[Q][SPT],
                                                const float (&g)[Q][SPT],
                                                float (&acc)[Q][Q], float (&gc)[Q][SPT]) {
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
#pragma unroll
    for (int j = 0; j < Q; ++j) gc[j][s] = 0.0f;
    if constexpr (!SOFT) {
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
          if constexpr (WANT_GC) gc[j][s] += w;
        }
      }
    } else {
      if (cf.ktrick) {
        float md = d[0][s];
#pragma unroll
        for (int j = 1; j < Q; ++j) md = fminf(md, d[j][s]);
        float u[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) u[j] = fast_exp2((md - d[j][s]) * a);
        float r[Q];
#pragma unroll
        for (int i = 0; i < Q; ++i) {
          float sm = cf.k[i][0] * u[0];
#pragma unroll
          for (int j = 1; j < Q; ++j) sm = fmaf(cf.k[i][j], u[j], sm);
          r[i] = g[i][s] * __builtin_amdgcn_rcpf(sm);
        }
#pragma unroll
        for (int i = 0; i < Q; ++i)
#pragma unroll
          for (int j = 0; j < Q; ++j) acc[i][j] = fmaf(r[i], u[j], acc[i][j]);
        if constexpr (WANT_GC) {
#pragma unroll
          for (int j = 0; j < Q; ++j) {
            float t = r[0] * cf.k[0][j];
#pragma unroll
            for (int i = 1; i < Q; ++i) t = fmaf(r[i], cf.k[i][j], t);
            gc[j][s] = u[j] * t;
          }
        }
      } else {
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
            if constexpr (WANT_GC) gc[j][s] += w;
          }
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
      score[s] = mn - bcoef * fast_log2(sm);
    }
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// --------------------------------------------------------------------------
// forward kernel
// --------------------------------------------------------------------------
template <int Q, int SPT, bool SOFT>
__global__ __launch_bounds__(kWave) void sankoff_fwd_kernel(
    const int4* __restrict__ steps, const int8_t* __restrict__ leaves,
    const float* __restrict__ cost, int n_int, int nl, int L, int tiles, float a, float bcoef,
    int hard_root, float* __restrict__ dp, float* __restrict__ site_score,
    double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tree = blockIdx.x / tiles;
  const int tile = blockIdx.x - tree * tiles;
  const int lane = threadIdx.x;
  const int site = (tile * kWave + lane) * SPT;
  const bool active = site < L;
  const int sc = active ? site : 0;

  Coef<Q> cf;
  load_coef<Q, SOFT>(cost, a, cf);

  const int4* prog = steps + (size_t)tree * n_int;
  const int8_t* lv = leaves + (size_t)tree * nl * L + sc;
  const size_t rowstride = (size_t)Q * L;
  float* dpt = dp ? dp + (size_t)tree * n_int * rowstride + sc : nullptr;

  float dv[Q][SPT];
  for (int k = 0; k < n_int; ++k) {
    const int4 stp = prog[k];
    float d[Q][SPT], m[Q][SPT];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int desc = c == 0 ? stp.y : stp.z;
      const int kind = (desc >> 24) & 3;
      if (kind == kKindLeaf) {
        leaf_rows<Q, SPT>(lv + (size_t)(desc & 0xFFFF) * L, d);
      } else if (kind == kKindInt) {
        lds_get<Q, SPT>(lds, (desc >> 16) & 0xFF, lane, d);
      } else {
        fill_sentinel<Q, SPT>(d);
      }
      message<Q, SPT, SOFT>(cf, a, bcoef, d, m);
#pragma unroll
      for (int i = 0; i < Q; ++i)
#pragma unroll
        for (int s = 0; s < SPT; ++s) dv[i][s] = (c == 0) ? m[i][s] : dv[i][s] + m[i][s];
    }
    const int row = stp.x & 0xFFFF;
    const int oslot = (stp.x >> 16) & 0xFF;
    if (dpt && active) {
#pragma unroll
      for (int i = 0; i < Q; ++i) st<SPT>(dpt + (size_t)row * rowstride + (size_t)i * L, dv[i]);
    }
    if (oslot != 0xFF) lds_put<Q, SPT>(lds, oslot, lane, dv);
  }
  // the root is the last step (plan.cpp)
  float score[SPT], w[Q][SPT];
  root_score<Q, SPT, SOFT>(dv, a, bcoef, hard_root != 0, score, w);
  double tot = 0.0;
  if (active) {
#pragma unroll
    for (int s = 0; s < SPT; ++s) tot += (double)score[s];
    if (site_score) st<SPT>(site_score + (size_t)tree * L + site, score);
  }
  tot = wave_sum(tot);
  if (lane == 0) part[blockIdx.x] = tot;
}

// --------------------------------------------------------------------------
// adjoint (reverse) kernel
// --------------------------------------------------------------------------
template <int Q, int SPT, bool SOFT>
__global__ __launch_bounds__(kWave) void sankoff_bwd_kernel(
    const int4* __restrict__ steps, const int8_t* __restrict__ leaves,
    const float* __restrict__ cost, int n_int, int nl, int L, int tiles, float a, float bcoef,
    int hard_root, const float* __restrict__ dp, const float* __restrict__ dts,
    float* __restrict__ marg, int8_t* __restrict__ anc, double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tree = blockIdx.x / tiles;
  const int tile = blockIdx.x - tree * tiles;
  const int lane = threadIdx.x;
  const int site = (tile * kWave + lane) * SPT;
  const bool active = site < L;
  const int sc = active ? site : 0;

  Coef<Q> cf;
  load_coef<Q, SOFT>(cost, a, cf);
  const float dscale = dts ? uniform(dts[tree]) : 1.0f;

  const int4* prog = steps + (size_t)tree * n_int;
  const int8_t* lv = leaves + (size_t)tree * nl * L + sc;
  const size_t rowstride = (size_t)Q * L;
  const float* dpt = dp + (size_t)tree * n_int * rowstride + sc;
  float* mt = marg ? marg + (size_t)tree * n_int * rowstride + sc : nullptr;
  int8_t* at = anc ? anc + (size_t)tree * n_int * L + sc : nullptr;

  float acc[Q][Q];
#pragma unroll
  for (int i = 0; i < Q; ++i)
#pragma unroll
    for (int j = 0; j < Q; ++j) acc[i][j] = 0.0f;

  for (int k = n_int - 1; k >= 0; --k) {
    const int4 stp = prog[k];
    if (stp.w & kStepUnreached) continue;
    const int row = stp.x & 0xFFFF;
    float g[Q][SPT];
    if (stp.w & kStepRoot) {
      float d[Q][SPT], score[SPT];
#pragma unroll
      for (int i = 0; i < Q; ++i) ld<SPT>(dpt + (size_t)row * rowstride + (size_t)i * L, d[i]);
      root_score<Q, SPT, SOFT>(d, a, bcoef, hard_root != 0, score, g);
      const float f = active ? dscale : 0.0f;
#pragma unroll
      for (int i = 0; i < Q; ++i)
#pragma unroll
        for (int s = 0; s < SPT; ++s) g[i][s] *= f;
    } else {
      lds_get<Q, SPT>(lds, (stp.x >> 16) & 0xFF, lane, g);
    }
    if (mt && active) {
#pragma unroll
      for (int i = 0; i < Q; ++i) st<SPT>(mt + (size_t)row * rowstride + (size_t)i * L, g[i]);
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
      st_codes<SPT>(at + (size_t)row * L, best);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int desc = c == 0 ? stp.y : stp.z;
      const int kind = (desc >> 24) & 3;
      float d[Q][SPT], gc[Q][SPT];
      if (kind == kKindLeaf) {
        leaf_rows<Q, SPT>(lv + (size_t)(desc & 0xFFFF) * L, d);
        message_adjoint<Q, SPT, SOFT, false>(cf, a, d, g, acc, gc);
      } else if (kind == kKindInt) {
        const int crow = desc & 0xFFFF;
#pragma unroll
        for (int j = 0; j < Q; ++j) ld<SPT>(dpt + (size_t)crow * rowstride + (size_t)j * L, d[j]);
        message_adjoint<Q, SPT, SOFT, true>(cf, a, d, g, acc, gc);
        const int cslot = (desc >> 16) & 0xFF;
        if (desc & kStepAccumulate) {
          float old[Q][SPT];
          lds_get<Q, SPT>(lds, cslot, lane, old);
#pragma unroll
          for (int j = 0; j < Q; ++j)
#pragma unroll
            for (int s = 0; s < SPT; ++s) gc[j][s] += old[j][s];
        }
        lds_put<Q, SPT>(lds, cslot, lane, gc);
      } else {
        fill_sentinel<Q, SPT>(d);
        message_adjoint<Q, SPT, SOFT, false>(cf, a, d, g, acc, gc);
      }
    }
  }
  double* out = part + (size_t)blockIdx.x * Q * Q;
#pragma unroll
  for (int i = 0; i < Q; ++i)
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const double v = wave_sum((double)acc[i][j]);
      if (lane == 0) out[i * Q + j] = v;
    }
}

// --------------------------------------------------------------------------
// trex-exact ancestral reconstruction (sankoff.py:166-185, 191-267)
// --------------------------------------------------------------------------
template <int Q, int SPT>
__global__ __launch_bounds__(kWave) void sankoff_backtrack_kernel(
    const int2* __restrict__ bt, const float* __restrict__ cost, const float* __restrict__ dp,
    int n_int, int L, int tiles, int8_t* __restrict__ anc) {
  const int tree = blockIdx.x / tiles;
  const int tile = blockIdx.x - tree * tiles;
  const int lane = threadIdx.x;
  const int site = (tile * kWave + lane) * SPT;
  if (site >= L) return;
  float c[Q][Q];
#pragma unroll
  for (int i = 0; i < Q; ++i)
#pragma unroll
    for (int j = 0; j < Q; ++j) c[i][j] = uniform(cost[i * Q + j]);
  const int2* prog = bt + (size_t)tree * n_int;
  const size_t rowstride = (size_t)Q * L;
  const float* dpt = dp + (size_t)tree * n_int * rowstride + site;
  int8_t* at = anc + (size_t)tree * n_int * L + site;
  for (int k = 0; k < n_int; ++k) {
    const int2 e = prog[k];
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
#pragma unroll
        for (int j = 0; j < Q; ++j) ld<SPT>(dpt + (size_t)x * rowstride + (size_t)j * L, d[j]);
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

// --------------------------------------------------------------------------
// reductions (fixed order => bitwise reproducible)
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void reduce_tree_kernel(const double* __restrict__ part,
                                                         int tiles, float* __restrict__ out) {
  __shared__ double sh[256];
  const int tree = blockIdx.x;
  double v = 0.0;
  for (int t = threadIdx.x; t < tiles; t += 256) v += part[(size_t)tree * tiles + t];
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[tree] = (float)sh[0];
}

template <int Q>
__global__ __launch_bounds__(256) void reduce_dcost_kernel(const double* __restrict__ part,
                                                          int nblocks, const float* __restrict__ cost,
                                                          float a, int soft, float* __restrict__ out) {
  __shared__ double sh[256];
  const int q = blockIdx.x;
  double v = 0.0;
  for (int t = threadIdx.x; t < nblocks; t += 256) v += part[(size_t)t * Q * Q + q];
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double f = 1.0;
    if (soft) {
      Coef<Q> cf;
      load_coef<Q, true>(cost, a, cf);
      if (cf.ktrick) f = (double)cf.k[q / Q][q % Q];
    }
    out[q] = (float)(sh[0] * f);
  }
}

// dp [B][n_int][Q][L] -> trex VmappedDPTable [B][L][n_all][Q]
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
      const float* src = dp + (((size_t)b * ni + (node - nl)) * Q) * L + l;
      for (int q = 0; q < Q; ++q) o[q] = src[(size_t)q * L];
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
  if (Q > 4)
    return set_error(TREX_E_UNSUPPORTED, "%s: Q=%d > 4 not supported by this build", fn, Q);
  sh->B = B;
  sh->L = L;
  sh->n_all = n_all;
  sh->nl = (n_all + 1) / 2;
  sh->ni = n_all - sh->nl;
  sh->Q = Q;
  return TREX_OK;
}

// sites per lane: widest that divides L and keeps the LDS stack <= 10 KiB per
// wave (>= 16 resident waves per CU); TREX_SPT overrides for tuning.
int pick_spt(int L, int n_slots, int Q) {
  static int forced = [] {
    const char* e = std::getenv("TREX_SPT");
    return e ? std::atoi(e) : 0;
  }();
  if (forced == 1 || forced == 2 || forced == 4) {
    if (L % forced == 0) return forced;
  }
  for (int s : {4, 2}) {
    if (L % s == 0 && (size_t)n_slots * Q * kWave * s * 4 <= 10240) return s;
  }
  return 1;
}

int tiles_for(int L, int spt) { return (L + kWave * spt - 1) / (kWave * spt); }

int hip_check(const char* fn) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

template <int Q, int SPT, bool SOFT>
void launch_fwd(const Shape& s, int tiles, size_t lds, hipStream_t st, const int4* steps,
                const int8_t* leaves, const float* cost, float a, float bcoef, int hard_root,
                float* dp, float* site_score, double* part) {
  hipLaunchKernelGGL((sankoff_fwd_kernel<Q, SPT, SOFT>), dim3(s.B * tiles), dim3(kWave), lds, st,
                     steps, leaves, cost, s.ni, s.nl, s.L, tiles, a, bcoef, hard_root, dp,
                     site_score, part);
}

template <int Q, int SPT, bool SOFT>
void launch_bwd(const Shape& s, int tiles, size_t lds, hipStream_t st, const int4* steps,
                const int8_t* leaves, const float* cost, float a, float bcoef, int hard_root,
                const float* dp, const float* dts, float* marg, int8_t* anc, double* part) {
  hipLaunchKernelGGL((sankoff_bwd_kernel<Q, SPT, SOFT>), dim3(s.B * tiles), dim3(kWave), lds, st,
                     steps, leaves, cost, s.ni, s.nl, s.L, tiles, a, bcoef, hard_root, dp, dts,
                     marg, anc, part);
}

template <int Q, bool SOFT>
void dispatch_fwd(int spt, const Shape& s, int tiles, size_t lds, hipStream_t st,
                  const int4* steps, const int8_t* leaves, const float* cost, float a, float bcoef,
                  int hr, float* dp, float* ss, double* part) {
  if (spt == 4)
    launch_fwd<Q, 4, SOFT>(s, tiles, lds, st, steps, leaves, cost, a, bcoef, hr, dp, ss, part);
  else if (spt == 2)
    launch_fwd<Q, 2, SOFT>(s, tiles, lds, st, steps, leaves, cost, a, bcoef, hr, dp, ss, part);
  else
    launch_fwd<Q, 1, SOFT>(s, tiles, lds, st, steps, leaves, cost, a, bcoef, hr, dp, ss, part);
}

template <int Q, bool SOFT>
void dispatch_bwd(int spt, const Shape& s, int tiles, size_t lds, hipStream_t st,
                  const int4* steps, const int8_t* leaves, const float* cost, float a, float bcoef,
                  int hr, const float* dp, const float* dts, float* marg, int8_t* anc,
                  double* part) {
  if (spt == 4)
    launch_bwd<Q, 4, SOFT>(s, tiles, lds, st, steps, leaves, cost, a, bcoef, hr, dp, dts, marg,
                           anc, part);
  else if (spt == 2)
    launch_bwd<Q, 2, SOFT>(s, tiles, lds, st, steps, leaves, cost, a, bcoef, hr, dp, dts, marg,
                           anc, part);
  else
    launch_bwd<Q, 1, SOFT>(s, tiles, lds, st, steps, leaves, cost, a, bcoef, hr, dp, dts, marg,
                           anc, part);
}

void tau_coefs(float tau, float* a, float* bcoef) {
  if (tau > 0.0f) {
    *a = (float)(1.4426950408889634 / (double)tau);
    *bcoef = (float)((double)tau * 0.6931471805599453);
  } else {
    *a = 0.0f;
    *bcoef = 0.0f;
  }
}

}  // namespace

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

}  // namespace trex

using namespace trex;

extern "C" const char* trex_last_error(void) { return g_err; }

extern "C" int trex_version(void) { return 1; }

extern "C" int64_t trex_workspace_bytes(int B, int L, int n_all, int Q) {
  if (B <= 0 || L <= 0 || Q <= 0) return 0;
  const int64_t nb = (int64_t)B * tiles_for(L, 1);
  return 256 + nb * 8 + nb * (int64_t)Q * Q * 8;
}

extern "C" int trex_sankoff_fwd(const int32_t* plan, int n_slots, const int8_t* leaves,
                                const float* cost, int B, int L, int n_all, int Q, float tau,
                                unsigned flags, float* dp, float* site_score, float* tree_score,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  Shape s;
  if (int e = check_shape("trex_sankoff_fwd", B, L, n_all, Q, &s)) return e;
  if (!plan || !leaves || !cost || !tree_score || !workspace)
    return set_error(TREX_E_ARG, "trex_sankoff_fwd: null pointer argument");
  if (!(tau >= 0.0f) || std::isinf(tau))
    return set_error(TREX_E_ARG, "trex_sankoff_fwd: tau must be finite and >= 0 (got %g)", tau);
  if (workspace_bytes < trex_workspace_bytes(B, L, n_all, Q))
    return set_error(TREX_E_ARG, "trex_sankoff_fwd: workspace too small");
  if (n_slots < 0 || n_slots > 250) return set_error(TREX_E_ARG, "trex_sankoff_fwd: bad n_slots");
  const int spt = pick_spt(L, n_slots, Q);
  const int tiles = tiles_for(L, spt);
  const size_t lds = (size_t)std::max(n_slots, 1) * Q * kWave * spt * sizeof(float);
  if (lds > 65536) return set_error(TREX_E_UNSUPPORTED, "trex_sankoff_fwd: LDS stack too deep");
  hipStream_t st = (hipStream_t)stream;
  const int4* steps = reinterpret_cast<const int4*>(plan + TREX_PLAN_HEADER_INTS);
  double* part = reinterpret_cast<double*>(workspace);
  float a, bc;
  tau_coefs(tau, &a, &bc);
  const int hr = (flags & TREX_FLAG_HARD_ROOT) ? 1 : 0;
  const bool soft = tau > 0.0f;
#define TREX_FWD(QQ)                                                                         \
  if (soft)                                                                                  \
    dispatch_fwd<QQ, true>(spt, s, tiles, lds, st, steps, leaves, cost, a, bc, hr, dp,       \
                           site_score, part);                                                \
  else                                                                                       \
    dispatch_fwd<QQ, false>(spt, s, tiles, lds, st, steps, leaves, cost, a, bc, hr, dp,      \
                            site_score, part);
  switch (Q) {
    case 2: TREX_FWD(2) break;
    case 3: TREX_FWD(3) break;
    case 4: TREX_FWD(4) break;
  }
#undef TREX_FWD
  if (int e = hip_check("trex_sankoff_fwd")) return e;
  hipLaunchKernelGGL(reduce_tree_kernel, dim3(B), dim3(256), 0, st, part, tiles, tree_score);
  return hip_check("trex_sankoff_fwd(reduce)");
}

extern "C" int trex_sankoff_bwd(const int32_t* plan, int n_slots, const int8_t* leaves,
                                const float* cost, int B, int L, int n_all, int Q, float tau,
                                unsigned flags, const float* dp, const float* d_tree_score,
                                float* d_cost, float* marginals, int8_t* anc_states,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  Shape s;
  if (int e = check_shape("trex_sankoff_bwd", B, L, n_all, Q, &s)) return e;
  if (!plan || !leaves || !cost || !dp || !d_cost || !workspace)
    return set_error(TREX_E_ARG, "trex_sankoff_bwd: null pointer argument");
  if (!(tau >= 0.0f) || std::isinf(tau))
    return set_error(TREX_E_ARG, "trex_sankoff_bwd: tau must be finite and >= 0 (got %g)", tau);
  if (workspace_bytes < trex_workspace_bytes(B, L, n_all, Q))
    return set_error(TREX_E_ARG, "trex_sankoff_bwd: workspace too small");
  if (n_slots < 0 || n_slots > 250) return set_error(TREX_E_ARG, "trex_sankoff_bwd: bad n_slots");
  const int spt = pick_spt(L, n_slots, Q);
  const int tiles = tiles_for(L, spt);
  const size_t lds = (size_t)std::max(n_slots, 1) * Q * kWave * spt * sizeof(float);
  if (lds > 65536) return set_error(TREX_E_UNSUPPORTED, "trex_sankoff_bwd: LDS stack too deep");
  hipStream_t st = (hipStream_t)stream;
  const int4* steps = reinterpret_cast<const int4*>(plan + TREX_PLAN_HEADER_INTS);
  double* part = reinterpret_cast<double*>(static_cast<char*>(workspace) + 256 +
                                           (int64_t)B * tiles_for(L, 1) * 8);
  float a, bc;
  tau_coefs(tau, &a, &bc);
  const int hr = (flags & TREX_FLAG_HARD_ROOT) ? 1 : 0;
  const bool soft = tau > 0.0f;
#define TREX_BWD(QQ)                                                                         \
  if (soft)                                                                                  \
    dispatch_bwd<QQ, true>(spt, s, tiles, lds, st, steps, leaves, cost, a, bc, hr, dp,       \
                           d_tree_score, marginals, anc_states, part);                       \
  else                                                                                       \
    dispatch_bwd<QQ, false>(spt, s, tiles, lds, st, steps, leaves, cost, a, bc, hr, dp,      \
                            d_tree_score, marginals, anc_states, part);                      \
  hipLaunchKernelGGL(reduce_dcost_kernel<QQ>, dim3(QQ * QQ), dim3(256), 0, st, part,           \
                     B * tiles, cost, a, soft ? 1 : 0, d_cost);
  switch (Q) {
    case 2: TREX_BWD(2) break;
    case 3: TREX_BWD(3) break;
    case 4: TREX_BWD(4) break;
  }
#undef TREX_BWD
  return hip_check("trex_sankoff_bwd");
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
  const int spt = (L % 4 == 0) ? 4 : 1;
  const int tiles = tiles_for(L, spt);
  hipStream_t st = (hipStream_t)stream;
  const int2* bt = reinterpret_cast<const int2*>(plan + TREX_PLAN_HEADER_INTS +
                                                 (int64_t)B * s.ni * 4);
#define TREX_BT(QQ)                                                                            \
  if (spt == 4)                                                                                \
    hipLaunchKernelGGL((sankoff_backtrack_kernel<QQ, 4>), dim3(B * tiles), dim3(kWave), 0, st, \
                       bt, cost, dp, s.ni, L, tiles, anc_states);                              \
  else                                                                                         \
    hipLaunchKernelGGL((sankoff_backtrack_kernel<QQ, 1>), dim3(B * tiles), dim3(kWave), 0, st, \
                       bt, cost, dp, s.ni, L, tiles, anc_states);
  switch (Q) {
    case 2: TREX_BT(2) break;
    case 3: TREX_BT(3) break;
    case 4: TREX_BT(4) break;
  }
#undef TREX_BT
  return hip_check("trex_sankoff_backtrack");
}

extern "C" int trex_dp_to_trex_layout(const float* dp, const int8_t* leaves, int B, int L,
                                      int n_all, int Q, float* out, void* stream) {
  Shape s;
  if (B <= 0 || L <= 0 || n_all < 3 || Q < 2 || !dp || !leaves || !out)
    return set_error(TREX_E_ARG, "trex_dp_to_trex_layout: bad arguments");
  s.nl = (n_all + 1) / 2;
  const size_t total = (size_t)B * n_all * L;
  const int grid = (int)std::min<size_t>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(to_trex_layout_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, dp,
                     leaves, B, L, n_all, s.nl, Q, out);
  return hip_check("trex_dp_to_trex_layout");
}
