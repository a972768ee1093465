// Device helpers shared by the Sankoff kernels (sankoff.hip: Q <= 4,
// sites-per-lane; sankoff_wide.hip: Q > 4, states-per-lane).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace trex {
namespace {

constexpr float kSentinel = 1e5f;  // sankoff.py:152
constexpr int kWave = 64;
constexpr int kKindLeaf = 1, kKindInt = 2;  // 0 = 1e5 sentinel row

// Read-only, wave-uniform data (topology program, cost matrix) goes through
// the constant address space so hipcc emits scalar loads (s_load): vector
// loads would be ordered behind the wave's in-flight DP-table stores in vmcnt.
template <class T>
using cptr = const __attribute__((address_space(4))) T*;
template <class T>
__device__ __forceinline__ cptr<T> as_const(const T* p) {
  return (cptr<T>)(p);
}

struct I4 {
  int x, y, z, w;
};
__device__ __forceinline__ I4 load_step(cptr<int> prog, int k) {
  return I4{prog[4 * k], prog[4 * k + 1], prog[4 * k + 2], prog[4 * k + 3]};
}

__device__ __forceinline__ float uniform(float x) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }

// SGPR cost-matrix modes: kHard (min-plus), kSoftK (factored softmin with
// K = exp(-(C - cmin)/tau)), kSoftDirect (per-row stabilised softmin, used
// when range(C)/tau > 40 would underflow K).
constexpr int kHard = 0, kSoftK = 1, kSoftDirect = 2;

// range(C)/tau <= 40: the factored form keeps every K >= e^-40
__device__ __forceinline__ bool use_ktrick(float cmin, float cmax, float a) {
  return (cmax - cmin) * a <= 57.70780f;  // log2(e^40)
}

// ---- buffer (SRD) access: 32-bit lane offset in voffset, row offset in
// soffset, no 64-bit VALU address arithmetic per access ----
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// ---- cross-lane sums without LDS: v_permlane32_swap / v_permlane16_swap
// (gfx950) for the two upper butterfly levels, DPP row / quad permutations
// inside a 16-lane row.  Fixed pairing: bitwise reproducible. ----
__device__ __forceinline__ double dbl(uint32_t lo, uint32_t hi) {
  return __hiloint2double((int)hi, (int)lo);
}
__device__ __forceinline__ uint32_t lo32(double v) { return (uint32_t)__double2loint(v); }
__device__ __forceinline__ uint32_t hi32(double v) { return (uint32_t)__double2hiint(v); }
// x, y -> (lanes < 32: x[l] + x[l + 32]; lanes >= 32: y[l - 32] + y[l])
__device__ __forceinline__ double swap32_add(double x, double y) {
  const auto a = __builtin_amdgcn_permlane32_swap(lo32(x), lo32(y), false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi32(x), hi32(y), false, false);
  return dbl(a[0], b[0]) + dbl(a[1], b[1]);
}
// x, y -> rows (16 lanes) 0, 2: x summed over row pairs (0,1), (2,3); rows 1, 3: y
__device__ __forceinline__ double swap16_add(double x, double y) {
  const auto a = __builtin_amdgcn_permlane16_swap(lo32(x), lo32(y), false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi32(x), hi32(y), false, false);
  return dbl(a[0], b[0]) + dbl(a[1], b[1]);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  return dbl((uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo32(v), CTRL, 0xF, 0xF, false),
             (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi32(v), CTRL, 0xF, 0xF, false));
}
constexpr int kDppRowRor8 = 0x128, kDppHalfMirror = 0x141, kDppQuadX1 = 0xB1, kDppQuadX2 = 0x4E;

// sum over the wave; lane 0 (every lane of quad 0, in fact) holds the total
__device__ __forceinline__ double wave_sum_lane0(double v) {
  v = swap32_add(v, v);
  v = swap16_add(v, v);
  v += dpp_d<kDppRowRor8>(v);
  v += dpp_d<kDppHalfMirror>(v);
  v += dpp_d<kDppQuadX2>(v);
  v += dpp_d<kDppQuadX1>(v);
  return v;
}

// reduce-scatter of 16 per-lane values: lane l returns the wave total of
// v[(l >> 2) & 15] (62 VALU ops instead of 16 full butterflies)
__device__ __forceinline__ double wave_reduce_scatter16(const double (&v)[16], int lane) {
  double w[8], z[4], y[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = swap32_add(v[k], v[k + 8]);  // index k + 8 (l >> 5)
#pragma unroll
  for (int k = 0; k < 4; ++k) z[k] = swap16_add(w[k], w[k + 4]);  // index k + 4 (l >> 4)
  const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // partner l ^ 8: index k + 2 b3 + 4 (l >> 4)
    const double keep = b3 ? z[k + 2] : z[k], send = b3 ? z[k] : z[k + 2];
    y[k] = keep + dpp_d<kDppRowRor8>(send);
  }
  // partner: the mirror lane in the 8-lane half row (opposite b2)
  const double keep = b2 ? y[1] : y[0], send = b2 ? y[0] : y[1];
  double x = keep + dpp_d<kDppHalfMirror>(send);
  x += dpp_d<kDppQuadX2>(x);
  x += dpp_d<kDppQuadX1>(x);
  return x;
}

__device__ __forceinline__ void store_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_sc1(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum of n values (lane-strided, fixed order) -> every lane
__device__ __forceinline__ double wave_sum_strided(const double* p, int n, int lane) {
  double v = 0.0;
  for (int t = lane; t < n; t += kWave) v += load_sc1(p + t);
  return wave_sum(v);
}

// packed FP32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes of work per VALU op)
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pk(float x, float y) { return f2{x, y}; }
__device__ __forceinline__ void pfma(float& d0, float& d1, f2 a, f2 b) {
  const f2 r = __builtin_elementwise_fma(a, b, f2{d0, d1});
  d0 = r.x;
  d1 = r.y;
}
// s = sum_j k[j] u[j] (pairs of j per packed op)
template <int Q>
__device__ __forceinline__ float kdot(const float (&krow)[Q], const float (&u)[Q]) {
  if constexpr (Q % 2 == 0) {
    f2 acc = pk(krow[0], krow[1]) * pk(u[0], u[1]);
#pragma unroll
    for (int j = 2; j < Q; j += 2) acc = __builtin_elementwise_fma(pk(krow[j], krow[j + 1]), pk(u[j], u[j + 1]), acc);
    return acc.x + acc.y;
  } else {
    float acc = krow[0] * u[0];
#pragma unroll
    for (int j = 1; j < Q; ++j) acc = fmaf(krow[j], u[j], acc);
    return acc;
  }
}
// acc[j] += r * v[j]
template <int Q>
__device__ __forceinline__ void axpy(float (&acc)[Q], float r, const float (&v)[Q]) {
  if constexpr (Q % 2 == 0) {
#pragma unroll
    for (int j = 0; j < Q; j += 2) pfma(acc[j], acc[j + 1], pk(r, r), pk(v[j], v[j + 1]));
  } else {
#pragma unroll
    for (int j = 0; j < Q; ++j) acc[j] = fmaf(r, v[j], acc[j]);
  }
}

}  // namespace
}  // namespace trex
