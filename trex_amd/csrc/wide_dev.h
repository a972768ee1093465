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

__host__ __device__ constexpr int wide_tab_floats(int G, int Q) { return (2 * Q + 1) * G; }

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
  float col[G];
  float cmin;
};

struct WLane {
  int lane, i, gbase;
  bool pad;  // state i >= Q
};

// message to parent state i:  min_j / smin_j (C[i][j] + D[j])   (sankoff.py:67-68)
template <int G, int MODE>
__device__ __forceinline__ float wmsg(const WCoef<G>& cf, float* X, const WLane& w, float a,
                                      float bcoef, float D) {
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
template <int G, int MODE>
__device__ __forceinline__ float wadj(const WCoef<G>& cf, float* X, const WLane& w, float a,
                                      float D, float g, float (&acc)[G]) {
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
    return u * kdot<G>(cf.col, rr);
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
    for (int p = 0; p < G; ++p) gc += (cf.col[p] + D == mm[p]) ? rr[p] : 0.0f;
    return gc;
  } else {
    float x[G];
    float mn = INFINITY;
#pragma unroll
    for (int j = 0; j < G; ++j) {
      x[j] = cf.row[j] + d[j];
      mn = fminf(mn, x[j]);
    }
    float e[G];
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < G; ++j) {
      e[j] = fast_exp2((mn - x[j]) * a);
      s += e[j];
    }
    const float r = w.pad ? 0.0f : g * __builtin_amdgcn_rcpf(s);
    axpy<G>(acc, r, e);
    float mm[G];
    xchg<G>(X + 2 * kWave, w.lane, w.gbase, r, rr);
    xchg<G>(X + 3 * kWave, w.lane, w.gbase, w.pad ? 0.0f : mn, mm);
    float gc = 0.0f;
#pragma unroll
    for (int p = 0; p < G; ++p) gc += rr[p] * fast_exp2((mm[p] - (cf.col[p] + D)) * a);
    return gc;
  }
}

// Fixed-order sum of n doubles by 256 threads (t = 0..255 of a group that
// owns red[256]); the result is in thread 0's return value.  Eight
// independent accumulators keep eight loads in flight per thread; the
// association is fixed, so the reduce kernel and the staged kernel's
// in-kernel tail give bitwise the same sums.  Every thread of the block
// must call it (it contains __syncthreads()).  COHERENT: device-scope loads
// (partials other workgroups wrote during the same launch).
template <bool COHERENT = false>
__device__ __forceinline__ double fixed_sum256(const double* src, int n, double* red, int t) {
  auto ld = [&](int k) { return COHERENT ? load_sc1(src + k) : src[k]; };
  double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int k = t;
  for (; k + 7 * 256 < n; k += 8 * 256) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += ld(k + j * 256);
  }
  for (; k < n; k += 256) acc[0] += ld(k);
  red[t] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h) red[t] += red[t + h];
    __syncthreads();
  }
  return red[0];
}

}  // namespace
}  // namespace trex
