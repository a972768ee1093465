// libtrexhip.so -- tree-cost kernels (maraxen/trex src/trex/tree.py) for gfx950.
//
//  a12 update_seq      (tree.py:110-130)  state softmax, fwd + VJP
//  a11 update_tree     (tree.py:50-107)   masked row softmax, fwd + VJP
//  a9  compute_surrogate_cost (tree.py:163-209): G = F F^T (MFMA f32, split-K),
//      loss / dA / M = diag(r+c) - (A+A^T) (one combine pass), dF = M F (MFMA)
//  a10 compute_soft_cost (tree.py:212-266): W = S C per site, G = F W^T
//  a13 enforce_graph_constraints (tree.py:133-160), fwd + grad
//  a8  compute_cost    (tree.py:269-296)  gather-reduce
//  a14 optax adam (+ clip_by_global_norm) fused update
//
// GEMMs run on v_mfma_f32_32x32x2_f32 (exact f32 fmaf chains; gfx950 has no
// reduced-precision f32 path).  All reductions are fixed-order (fp64), so
// results are bitwise reproducible.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "sankoff_dev.h"
#include "trex_common.h"


namespace trex {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

int tree_hip_check(const char* fn) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

__device__ __forceinline__ double block_sum_256(double v, double* sh) {
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------
// a12 update_seq: S = softmax_q(T * X) per (ancestor, site)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void update_seq_kernel(const float* __restrict__ x, int64_t rows,
                                                        int Q, float T, float* __restrict__ s) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool al = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(s)) & 15) == 0;
  if (Q == 4 && al) {  // one float4 in, one float4 out per row
    const float4* x4 = reinterpret_cast<const float4*>(x);
    float4* s4 = reinterpret_cast<float4*>(s);
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += stride) {
      const float4 v = x4[r];
      const float a = v.x * T, b = v.y * T, c = v.z * T, d = v.w * T;
      const float m = fmaxf(fmaxf(a, b), fmaxf(c, d));
      const float ea = expf(a - m), eb = expf(b - m), ec = expf(c - m), ed = expf(d - m);
      const float inv = 1.0f / (((ea + eb) + ec) + ed);
      s4[r] = make_float4(ea * inv, eb * inv, ec * inv, ed * inv);
    }
    return;
  }
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += stride) {
    const float* xr = x + r * Q;
    float* sr = s + r * Q;
    float m = -INFINITY;
    for (int q = 0; q < Q; ++q) m = fmaxf(m, xr[q] * T);
    float sum = 0.0f;
    for (int q = 0; q < Q; ++q) sum += expf(xr[q] * T - m);
    const float inv = 1.0f / sum;
    for (int q = 0; q < Q; ++q) sr[q] = expf(xr[q] * T - m) * inv;  // one store per element
  }
}

__global__ __launch_bounds__(256) void update_seq_bwd_kernel(const float* __restrict__ s,
                                                            const float* __restrict__ ds,
                                                            int64_t rows, int Q, float T,
                                                            float* __restrict__ dx) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool al = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(ds) |
                    reinterpret_cast<uintptr_t>(dx)) & 15) == 0;
  if (Q == 4 && al) {
    const float4* s4 = reinterpret_cast<const float4*>(s);
    const float4* g4 = reinterpret_cast<const float4*>(ds);
    float4* d4 = reinterpret_cast<float4*>(dx);
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += stride) {
      const float4 a = s4[r], g = g4[r];
      float dot = a.x * g.x;
      dot = fmaf(a.y, g.y, dot);
      dot = fmaf(a.z, g.z, dot);
      dot = fmaf(a.w, g.w, dot);
      d4[r] = make_float4(T * a.x * (g.x - dot), T * a.y * (g.y - dot), T * a.z * (g.z - dot),
                          T * a.w * (g.w - dot));
    }
    return;
  }
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += stride) {
    const float* sr = s + r * Q;
    const float* gr = ds + r * Q;
    float dot = 0.0f;
    for (int q = 0; q < Q; ++q) dot = fmaf(sr[q], gr[q], dot);
    for (int q = 0; q < Q; ++q) dx[r * Q + q] = T * sr[q] * (gr[q] - dot);
  }
}

// ---------------------------------------------------------------------------
// a11 update_tree: logits z (masked), A = row softmax.  One block per row.
//   theta/noise/gates [N-1][n_anc]; A [N][N]
// ---------------------------------------------------------------------------
__device__ __forceinline__ float tree_logit(const float* theta, const float* noise,
                                            const float* gates, int N, int n_anc, float T, int i,
                                            int j, bool* valid) {
  const int nl = N - n_anc;
  *valid = false;
  if (i == N - 1) {
    if (j == N - 1) { *valid = true; return 1.0f; }
    return -INFINITY;
  }
  if (j < nl) return -INFINITY;
  const int ja = j - nl;
  if (i >= nl && !(ja > i - nl)) return -INFINITY;  // ancestor block: upper triangular
  const size_t k = (size_t)i * n_anc + ja;
  float p = theta[k] + (noise ? noise[k] : 0.0f);
  if (gates) p *= gates[k];
  *valid = true;
  return p / T;
}

__global__ __launch_bounds__(256) void update_tree_kernel(const float* __restrict__ theta,
                                                         const float* __restrict__ noise,
                                                         const float* __restrict__ gates, int N,
                                                         int n_anc, float T, float* __restrict__ A) {
  __shared__ float red[256];
  const int i = blockIdx.x;
  float m = -INFINITY;
  for (int j = threadIdx.x; j < N; j += 256) {
    bool v;
    m = fmaxf(m, tree_logit(theta, noise, gates, N, n_anc, T, i, j, &v));
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  m = red[0];
  __syncthreads();
  float s = 0.0f;
  for (int j = threadIdx.x; j < N; j += 256) {
    bool v;
    const float z = tree_logit(theta, noise, gates, N, n_anc, T, i, j, &v);
    const float e = v ? expf(z - m) : 0.0f;
    A[(size_t)i * N + j] = e;
    s += e;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float inv = 1.0f / red[0];
  for (int j = threadIdx.x; j < N; j += 256) A[(size_t)i * N + j] *= inv;
}

__global__ __launch_bounds__(256) void update_tree_bwd_kernel(const float* __restrict__ A,
                                                             const float* __restrict__ dA,
                                                             const float* __restrict__ gates,
                                                             int N, int n_anc, float T,
                                                             float* __restrict__ dtheta) {
  __shared__ double sh[256];
  const int i = blockIdx.x;  // rows 0..N-2
  const int nl = N - n_anc;
  double dot = 0.0;
  for (int j = threadIdx.x; j < N; j += 256)
    dot += (double)A[(size_t)i * N + j] * (double)dA[(size_t)i * N + j];
  const float d = (float)block_sum_256(dot, sh);
  for (int ja = threadIdx.x; ja < n_anc; ja += 256) {
    const int j = nl + ja;
    const bool valid = (i < nl) || (ja > i - nl);
    float g = 0.0f;
    if (valid) {
      const float a = A[(size_t)i * N + j];
      g = a * (dA[(size_t)i * N + j] - d) / T;
      if (gates) g *= gates[(size_t)i * n_anc + ja];
    }
    dtheta[(size_t)i * n_anc + ja] = g;
  }
}

// ---------------------------------------------------------------------------
// a9 Gram G = X Y^T on MFMA f32 (X, Y: [N][K] row-major).  One wave computes
// a 64x64 tile (2x2 32x32 accumulators) over one K slice.  Lane l (row
// r = l&31, half h = l>>5) loads 16 consecutive k of its row per fragment;
// MFMA t then covers k = kb + t and kb + 16 + t on the two halves (the k
// permutation is the same for X and Y, so the dot products are exact).
// Blocks are grouped so that one XCD (blockIdx % 8) walks the tiles of one
// K slice while that slice is L2-resident.
// ---------------------------------------------------------------------------
// 16 consecutive k of one row (row stride K), zero past kend / nrows
__device__ __forceinline__ void load_frag16(const float* __restrict__ base, int row, int nrows,
                                            int K, int k0, int kend, float (&o)[16]) {
  if (row < nrows && k0 + 16 <= kend && (K & 3) == 0) {
    const float4* p = reinterpret_cast<const float4*>(base + (size_t)row * K + k0);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 v = p[t];
      o[4 * t] = v.x; o[4 * t + 1] = v.y; o[4 * t + 2] = v.z; o[4 * t + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < 16; ++t)
      o[t] = (row < nrows && k0 + t < kend) ? base[(size_t)row * K + k0 + t] : 0.0f;
  }
}

// pair -> (ti, tj).  symmetric: the upper triangle (ti <= tj) row-major,
// minus the tiles with both ti, tj < t0 (a cached constant block, e.g. the
// fixed leaf x leaf Gram of the C5 loop)
__host__ __device__ __forceinline__ int sym_row_len(int a, int ntile, int t0) {
  return ntile - (a > t0 ? a : t0);
}
__device__ __forceinline__ void pair_tiles(int pair, int ntile, int symmetric, int t0, int* ti,
                                           int* tj) {
  if (symmetric) {
    int a = 0, rem = pair;
    while (rem >= sym_row_len(a, ntile, t0)) { rem -= sym_row_len(a, ntile, t0); ++a; }
    *ti = a;
    *tj = (a > t0 ? a : t0) + rem;
  } else {
    *ti = pair / ntile;
    *tj = pair % ntile;
  }
}

__global__ __launch_bounds__(kWave) void gram_kernel(const float* __restrict__ X,
                                                    const float* __restrict__ Y, int N, int K,
                                                    int ntile, int npairs, int symmetric, int t0,
                                                    int ksplit, int kslice,
                                                    float* __restrict__ part) {
  const int b = blockIdx.x;
  const int xcd = b & 7, m = b >> 3;
  const int split = (m / npairs) * 8 + xcd;
  const int pair = m % npairs;
  if (split >= ksplit) return;
  int ti, tj;
  pair_tiles(pair, ntile, symmetric, t0, &ti, &tj);
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const int k_lo = split * kslice, k_hi = min(K, k_lo + kslice);
  f32x16 acc[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[u][v] = (f32x16){};
  for (int kb = k_lo; kb < k_hi; kb += 32) {
    float xa[2][16], yb[2][16];
#pragma unroll
    for (int u = 0; u < 2; ++u) load_frag16(X, ti * 64 + u * 32 + r, N, K, kb + 16 * h, k_hi, xa[u]);
#pragma unroll
    for (int v = 0; v < 2; ++v) load_frag16(Y, tj * 64 + v * 32 + r, N, K, kb + 16 * h, k_hi, yb[v]);
#pragma unroll
    for (int t = 0; t < 16; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v)
          acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[u][t], yb[v][t], acc[u][v], 0, 0, 0);
  }
  // partial tile [split][pair][64][64]
  float* out = part + ((size_t)split * npairs + pair) * 64 * 64;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
        out[(u * 32 + row) * 64 + v * 32 + r] = acc[u][v][q];
      }
}

// v2 Gram: k step 16 per fragment, the next step's fragments requested
// before this step's MFMAs (ping-pong registers, loop unrolled by two so
// nothing is copied).  Lane (r, h) loads X[row][kb + 8h .. kb + 8h + 8)
// (two float4); MFMA t covers k = kb + t (h = 0) and kb + 8 + t (h = 1).
// Loads are unconditional (clamped row, zero select) so every path issues
// the same VMEM ops.  Needs K % 16 == 0 and kslice % 32 == 0.
struct Frag8 {
  float v[2][8];
};
__device__ __forceinline__ void load_rows8(const float* __restrict__ base, int row0, int nrows,
                                           int K, int k0, float (&o)[2][8]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int row = row0 + u * 32;
    const bool ok = row < nrows;
    const float4* p = reinterpret_cast<const float4*>(base + (size_t)(ok ? row : 0) * K + k0);
    const float4 a = p[0], b = p[1];
    o[u][0] = ok ? a.x : 0.0f; o[u][1] = ok ? a.y : 0.0f; o[u][2] = ok ? a.z : 0.0f;
    o[u][3] = ok ? a.w : 0.0f; o[u][4] = ok ? b.x : 0.0f; o[u][5] = ok ? b.y : 0.0f;
    o[u][6] = ok ? b.z : 0.0f; o[u][7] = ok ? b.w : 0.0f;
  }
}

// ---- f16x3 split products (X3 variants) --------------------------------
// x*s = hi + lo with hi = f16(x*s), lo = f16(x*s - hi): 22 significant bits;
// x*y ~ hi_x hi_y + hi_x lo_y + lo_x hi_y (lo_x lo_y, ~2^-22 relative, and
// the split residuals dropped) on v_mfma_f32_32x32x16_f16 with f32
// accumulation: 3 f16 MFMAs (96 cycles/SIMD) replace 8 f32 ones (512) per
// 32x32x16 block.  The power-of-two operand scales keep |x*s| <= 2^14 (no
// f16 overflow) and lo out of the f16 subnormal range; the result is scaled
// back exactly.  Error per product <~ 1e-6 relative, random in sign: the
// tests hold these GEMMs to the same rtol 1e-5 vs fp64 as the f32 path.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void split_h8(const float (&x)[8], float scale, h8& hi, h8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = x[j] * scale;
    const _Float16 h = (_Float16)v;
    hi[j] = h;
    lo[j] = (_Float16)(v - (float)h);
  }
}
__device__ __forceinline__ f32x16 mfma_x3(const h8& ah, const h8& al, const h8& bh, const h8& bl,
                                          f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
}

// X3: f16x3 split products; sx, sy operand scales, out scaled by 1/(sx sy)
template <bool X3>
__global__ __launch_bounds__(kWave) void gram_kernel2(const float* __restrict__ X,
                                                     const float* __restrict__ Y, int N, int K,
                                                     int ntile, int npairs, int symmetric, int t0,
                                                     int ksplit, int kslice,
                                                     float* __restrict__ part, float sx = 1.0f,
                                                     float sy = 1.0f) {
  const int b = blockIdx.x;
  const int xcd = b & 7, m = b >> 3;
  const int split = (m / npairs) * 8 + xcd;
  const int pair = m % npairs;
  if (split >= ksplit) return;
  int ti, tj;
  pair_tiles(pair, ntile, symmetric, t0, &ti, &tj);
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const int k_lo = split * kslice, k_hi = min(K, k_lo + kslice);
  f32x16 acc[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[u][v] = (f32x16){};
  const int xr = ti * 64 + r, yr = tj * 64 + r;
  auto fetch = [&](int kb, float (&xa)[2][8], float (&yb)[2][8]) {
    const int k0 = min(kb, K - 16) + 8 * h;  // past k_hi: a valid address, product masked below
    load_rows8(X, xr, N, K, k0, xa);
    load_rows8(Y, yr, N, K, k0, yb);
  };
  auto compute = [&](int kb, float (&xa)[2][8], float (&yb)[2][8]) {
    if (kb >= k_hi) return;
    if constexpr (X3) {
      // lane (r, h) holds A[row r][k = 8h + j] and B[k = 8h + j][col r]: the
      // 32x32x16 f16 fragments are exactly the loaded 8-float runs
      h8 xh[2], xl[2], yh[2], yl[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) split_h8(xa[u], sx, xh[u], xl[u]);
#pragma unroll
      for (int v = 0; v < 2; ++v) split_h8(yb[v], sy, yh[v], yl[v]);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) acc[u][v] = mfma_x3(xh[u], xl[u], yh[v], yl[v], acc[u][v]);
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int v = 0; v < 2; ++v)
            acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[u][t], yb[v][t], acc[u][v], 0, 0, 0);
    }
  };
  float xa0[2][8], yb0[2][8], xa1[2][8], yb1[2][8];
  fetch(k_lo, xa0, yb0);
  for (int kb = k_lo; kb < k_hi; kb += 32) {
    fetch(kb + 16, xa1, yb1);
    compute(kb, xa0, yb0);
    fetch(kb + 32, xa0, yb0);
    compute(kb + 16, xa1, yb1);
  }
  const float unscale = X3 ? 1.0f / (sx * sy) : 1.0f;
  float* out = part + ((size_t)split * npairs + pair) * 64 * 64;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
        out[(u * 32 + row) * 64 + v * 32 + r] = acc[u][v][q] * unscale;
      }
}

// G[i][j] = sum over splits (fixed order, fp64); symmetric tiles mirrored
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ part, int N,
                                                         int ntile, int npairs, int ksplit,
                                                         int symmetric, int t0,
                                                         float* __restrict__ G) {
  const size_t total = (size_t)npairs * 4096;
  for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (size_t)gridDim.x * 256) {
    const int pair = (int)(t / 4096);
    const int e = (int)(t % 4096);
    int ti, tj;
    pair_tiles(pair, ntile, symmetric, t0, &ti, &tj);
    double s = 0.0;
    for (int sp = 0; sp < ksplit; ++sp) s += (double)part[((size_t)sp * npairs + pair) * 4096 + e];
    const int i = ti * 64 + e / 64, j = tj * 64 + e % 64;
    // a diagonal tile holds both (i, j) and (j, i): only i <= j writes the
    // pair, or two threads would race on it with differently rounded sums
    if (i < N && j < N && (!symmetric || ti != tj || i <= j)) {
      G[(size_t)i * N + j] = (float)s;
      if (symmetric) G[(size_t)j * N + i] = (float)s;
    }
  }
}

// ---- v3 Gram: LDS-staged K chunks, one workgroup per CU -------------------
// Symmetric G = S S^T (f16x3 split products) over the needed 32x32 tiles:
// the upper triangle minus the cached leaf x leaf block (tiles with both
// strips < t0s), enumerated row-major like pair_tiles.  A workgroup is 8
// waves, two per SIMD (256 registers each, no spills): a wave owns up to 13
// tiles (208 accumulator registers); a workgroup owns up to 104 tiles (a
// "group"; more tiles -> more groups; C5's 100 tiles are one) and a
// contiguous range of 16-wide K chunks (its split), one workgroup per CU.
// Per chunk all N <= 512 rows are loaded ONCE from HBM (one dwordx4 per
// thread per 128 rows, issued a chunk ahead into
// registers), split into f16 hi / lo planes in LDS (double-buffered, row
// stride 80 B: hi k0..15 | lo k0..15 | pad), and every wave feeds its
// tiles' 32x32x16 MFMAs from LDS fragments (the A fragment re-read only when
// the tile row strip changes).  The v2 kernel instead re-read each row once
// per 64x64 tile pair from L2 with one wave per pair: load-bound.
// Partials [split][tile][32][32] (scaled back) reduce in a fixed order.
constexpr int kG3Rows = 512;
constexpr int kG3Stride = 80;
constexpr int kG3Tiles = 13;
constexpr int kG3Waves = 8;
constexpr int kG3Rows4 = kG3Waves * 64 / 4;  // rows per load pass (128)
constexpr int kG3Buf = kG3Rows * kG3Stride;
constexpr int kG3Lds = 2 * kG3Buf;

typedef _Float16 h4 __attribute__((ext_vector_type(4)));

// workgroup barrier for LDS hand-over only: waits for this wave's LDS ops
// (lgkmcnt) but NOT for its outstanding global loads -- __syncthreads()'s
// fence would drain vmcnt and so the register prefetch of the next chunk
// at every barrier
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// f16x3 operand pre-split (x3p entry points, trex_tree_split_x3): every
// group of 4 consecutive f32 values x * s is stored as 16 bytes -- the four
// f16 hi parts, then the four f16 lo parts -- so a 16-B load of the
// pre-split operand lands at the same byte offset as the f32 one and the
// kernels stage it into LDS without the split arithmetic
__device__ __forceinline__ u32x4 split_x3_group(float x0, float x1, float x2, float x3, float s) {
  const float v[4] = {x0 * s, x1 * s, x2 * s, x3 * s};
  h4 hi, lo;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hi[j] = (_Float16)v[j];
    lo[j] = (_Float16)(v[j] - (float)hi[j]);
  }
  const uint2 a = __builtin_bit_cast(uint2, hi), b = __builtin_bit_cast(uint2, lo);
  return (u32x4){a.x, a.y, b.x, b.y};
}

template <bool PRE = false>
__device__ __forceinline__ void g3_stage(unsigned char* buf, int row, int sub, const u32x4& w,
                                         float sc) {
  if constexpr (PRE) {
    *reinterpret_cast<uint2*>(buf + row * kG3Stride + sub * 8) = uint2{w.x, w.y};
    *reinterpret_cast<uint2*>(buf + row * kG3Stride + 32 + sub * 8) = uint2{w.z, w.w};
    return;
  }
  const float v[4] = {__uint_as_float(w.x) * sc, __uint_as_float(w.y) * sc,
                      __uint_as_float(w.z) * sc, __uint_as_float(w.w) * sc};
  h4 hi, lo;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hi[j] = (_Float16)v[j];
    lo[j] = (_Float16)(v[j] - (float)hi[j]);
  }
  *reinterpret_cast<h4*>(buf + row * kG3Stride + sub * 8) = hi;
  *reinterpret_cast<h4*>(buf + row * kG3Stride + 32 + sub * 8) = lo;
}

// NCP (PRE only): rows [0, 128 NCP) -- the first NCP row passes -- are exact
// one-hot leaf rows read as their code bytes (codes, trex_tree_leaf_codes;
// one byte per site instead of a 16-B pre-split piece) and expanded into
// the same f16 image (hi = one-hot x sc, lo = 0): bitwise the pre-split rows.
// The pass split is compile-time: a runtime per-row choice spilled (11-16
// VGPRs) and cost the whole kernel 1.7x
template <bool PRE = false, int NCP = 0>  // PRE: S pre-split (split_x3_group layout)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void gram_kernel3(
    const float* __restrict__ S, int N, int K, int ns, int t0s, int ntiles, int ngroups,
    int ksplit, int nchunks, float sc, float* __restrict__ part, int lzs = 0,
    const uint8_t* __restrict__ codes = nullptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds3[];
  const int g = blockIdx.x % ngroups;
  const int split = blockIdx.x / ngroups;
  const int c_lo = (int)((int64_t)split * nchunks / ksplit);
  const int c_hi = (int)((int64_t)(split + 1) * nchunks / ksplit);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int tb = (g * kG3Waves + wave) * kG3Tiles;
  const int nt = max(0, min(kG3Tiles, ntiles - tb));
  // first tile's strips; tiles past the wave's range (t >= nt) run on
  // whatever strips follow (clamped to ns - 1) and are not written: every
  // wave issues the same unconditional MFMA stream.  (Spreading the leaf
  // strips' 2-MFMA tiles evenly over the SIMDs measured no gain, PERFLOG.)
  int a0, b0;
  pair_tiles(min(tb, ntiles - 1), ns, 1, t0s, &a0, &b0);

  f32x16 acc[kG3Tiles];
#pragma unroll
  for (int t = 0; t < kG3Tiles; ++t) acc[t] = (f32x16){};

  // loads: thread (rb = tid / 4, sub = tid % 4) fetches S[rb + 128 i][k0 + 4 sub .. + 4);
  // rows past N read out of bounds (0)
  const rsrc_t rs = make_rsrc(S, (uint32_t)((size_t)N * K * 4));
  const int sub = tid & 3, rb = tid >> 2;
  constexpr int kRowsPerPass = kG3Waves * kWave / 4;
  static_assert(NCP == 0 || PRE, "code rows need the pre-split image");
  u32x4 pf[kG3Rows / kRowsPerPass - NCP];
  uint32_t pcode[NCP > 0 ? NCP : 1];
  const rsrc_t rcd = make_rsrc(codes, (uint32_t)((size_t)kRowsPerPass * NCP * (K / 4)));
  auto gload = [&](int c) {
#pragma unroll
    for (int i = 0; i < kG3Rows / kRowsPerPass; ++i) {
      const int vo = ((rb + kRowsPerPass * i) * K + 4 * sub) * 4;  // code byte: vo / 16
      if (i < NCP)
        pcode[i < NCP ? i : 0] = __builtin_amdgcn_raw_buffer_load_b8(rcd, vo >> 4, c * 4, 0);
      else
        pf[i - NCP] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, c * 64, 0);
    }
  };
  const uint32_t hb = (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)sc);  // one-hot 1 x sc
  // K % 16 != 0 (K % 4 == 0): the last chunk's columns past K hold the next
  // row's first values (or read out of bounds: 0); staged as zeros, they add
  // nothing to any product
  auto stage = [&](unsigned char* buf, int c) {
    const bool kv = 16 * c + 4 * sub < K;
#pragma unroll
    for (int i = 0; i < kG3Rows / kRowsPerPass; ++i)
    {
      const int row = rb + kRowsPerPass * i;
      if (i < NCP) {
        const uint32_t code = kv ? (pcode[i < NCP ? i : 0] & 0xFFu) : 0xFFu;
        const u32x4 w = {(code == 0 ? hb : 0u) | ((code == 1 ? hb : 0u) << 16),
                         (code == 2 ? hb : 0u) | ((code == 3 ? hb : 0u) << 16), 0u, 0u};
        g3_stage<true>(buf, row, sub, w, sc);
      } else {
        g3_stage<PRE>(buf, row, sub, kv ? pf[i - NCP] : (u32x4){0u, 0u, 0u, 0u}, sc);
      }
    }
  };
  const int lofs = r * kG3Stride + 16 * h;
  auto compute = [&](const unsigned char* buf) {
    int a = a0, b = b0, ap = -1;
    h8 ah, al;
    // B fragments one tile ahead: tile t + 1's reads are issued before tile
    // t's MFMAs (the A fragment only when the row strip changes: a wave's
    // 13 tiles span 2-3 strips; LDS read bytes per chunk 416 -> ~240 KB per CU)
    h8 bh = *reinterpret_cast<const h8*>(buf + b * (32 * kG3Stride) + lofs);
    h8 bl = *reinterpret_cast<const h8*>(buf + b * (32 * kG3Stride) + lofs + 32);
#pragma unroll
    for (int t = 0; t < kG3Tiles; ++t) {
      // strips a < lzs: exact one-hot leaf rows, whose lo plane is zero
      const bool zlo = a < lzs;
      if (a != ap) {
        const unsigned char* pa = buf + a * (32 * kG3Stride) + lofs;
        ah = *reinterpret_cast<const h8*>(pa);
        al = *reinterpret_cast<const h8*>(pa + 32);
        ap = a;
      }
      const bool wrap = b + 1 >= ns;
      const int an = wrap ? min(a + 1, ns - 1) : a;
      const int bn = wrap ? (an > t0s ? an : t0s) : b + 1;
      h8 bhn = bh, bln = bl;
      if (t + 1 < kG3Tiles) {
        const unsigned char* pb = buf + bn * (32 * kG3Stride) + lofs;
        bhn = *reinterpret_cast<const h8*>(pb);
        bln = *reinterpret_cast<const h8*>(pb + 32);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch reads above the MFMAs
      // a zero lo plane adds exact zeros: its MFMA is skipped (bitwise)
      if (!zlo) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[t], 0, 0, 0);
      bh = bhn;
      bl = bln;
      a = an;
      b = bn;
    }
  };

  if (c_lo < c_hi) {
    gload(c_lo);
    stage(lds3, c_lo);
    if (c_lo + 1 < c_hi) gload(c_lo + 1);
  }
  lds_barrier();
  for (int c = c_lo; c < c_hi; ++c) {
    unsigned char* cb = lds3 + ((c - c_lo) & 1) * kG3Buf;
    unsigned char* nb = lds3 + (((c - c_lo) & 1) ^ 1) * kG3Buf;
    compute(cb);
    if (c + 1 < c_hi) {
      stage(nb, c + 1);
      if (c + 2 < c_hi) gload(c + 2);
    }
    lds_barrier();
  }

  const float unscale = 1.0f / (sc * sc);
#pragma unroll
  for (int t = 0; t < kG3Tiles; ++t) {
    if (t < nt) {
      float* out = part + ((size_t)split * ntiles + tb + t) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
        out[row * 32 + r] = acc[t][q] * unscale;
      }
    }
  }
}

// G[i][j] = G[j][i] = sum over splits of the v3 partials, fp64 in a fixed
// association: thread (e, q) of a block (64 elements x 4 quarters) sums the
// splits sp = q, q + 4, ... in order (4 independent loads in flight), then
// the four quarter sums add in q order.  One wave reads 256 contiguous bytes
// per split; the grid has ntiles * 16 waves (the serial one-thread-per-
// element loop kept too few loads in flight: 1.4 TB/s).
__global__ __launch_bounds__(256) void gram3_reduce_kernel(const float* __restrict__ part, int N,
                                                          int ns, int t0s, int ntiles,
                                                          int ksplit, float* __restrict__ G) {
  __shared__ double qs[4][64];
  const int el = threadIdx.x & 63, q = threadIdx.x >> 6;
  const size_t t = (size_t)blockIdx.x * 64 + el;  // element index, < ntiles * 1024
  const size_t stride = (size_t)ntiles * 1024;
  const float* src = part + t;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int sp = q;
  for (; sp + 12 < ksplit; sp += 16) {
    s0 += (double)src[(size_t)sp * stride];
    s1 += (double)src[(size_t)(sp + 4) * stride];
    s2 += (double)src[(size_t)(sp + 8) * stride];
    s3 += (double)src[(size_t)(sp + 12) * stride];
  }
  for (; sp < ksplit; sp += 4) s0 += (double)src[(size_t)sp * stride];
  qs[q][el] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (q != 0) return;
  const double s = ((qs[0][el] + qs[1][el]) + qs[2][el]) + qs[3][el];
  const int tile = (int)(t >> 10);
  const int e = (int)(t & 1023);
  int si, sj;
  pair_tiles(tile, ns, 1, t0s, &si, &sj);
  const int i = si * 32 + (e >> 5), j = sj * 32 + (e & 31);
  // diagonal tiles: only i <= j writes the mirrored pair (no write race)
  if (i < N && j < N && (si != sj || i <= j)) {
    G[(size_t)i * N + j] = (float)s;
    G[(size_t)j * N + i] = (float)s;
  }
}

// ---- v5 Gram: one wave per SIMD, software-pipelined fragment reads ---------
// v3's tile enumeration and staging, re-shaped for the MFMA pipe (v3 lost
// ~60 % of it: every tile's fragments were read right before its MFMAs behind
// an lgkmcnt(0), and the A-fragment reuse branch split the loop into one
// basic block per tile).  Here a workgroup is 4 waves (one per SIMD, up to
// 512 registers: the accumulators live in AGPRs); a wave owns T <= 16
// consecutive tiles and reads tile t + 1's A / B fragments (4 ds_read_b128)
// while tile t's three MFMAs run -- no branch anywhere in the chunk body, so
// the per-row f16 staging of the next chunk and the global loads of the
// chunk after it are interleaved between the MFMAs (row i of the stage after
// tile i; raw rows one chunk ahead in registers).
// A workgroup holds at most 64 tiles, so C5's 100 tiles take two groups; the
// two groups of a K split sit on the same XCD (blockIdx % 8) and run at the
// same pace, so the second read of each chunk is an L2 hit.
// X3 = false: the exact f32 Gram on v_mfma_f32_32x32x2_f32 -- rows staged as
// f32 (the same 80-B row stride), a lane's 8 k of a fragment (k = 8h .. 8h +
// 7) read as two float4 and fed to 8 MFMAs (MFMA t covers k = t and 8 + t on
// the two lane halves: the same permutation for both operands).
constexpr int kG5Waves = 4;
constexpr int kG5MaxTiles = 16;

typedef float f32x8 __attribute__((ext_vector_type(8)));

// W = 8 (two waves per SIMD, T <= 8 tiles each: 128 accumulator registers)
// is the x3 variant under test (TREX_GRAM=6)
template <int T, bool X3, int W = kG5Waves>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(W / 4, W / 4))) void gram_kernel5(
    const float* __restrict__ S, int N, int K, int ns, int t0s, int ntiles, int ngroups,
    int ksplit, int nchunks, float sc, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds5[];
  const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
  const int g = m % ngroups;
  const int split = (m / ngroups) * 8 + xcd;
  if (split >= ksplit) return;
  const int c_lo = (int)((int64_t)split * nchunks / ksplit);
  const int c_hi = (int)((int64_t)(split + 1) * nchunks / ksplit);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int tb = (g * W + wave) * T;
  const int nt = max(0, min(T, ntiles - tb));
  // per-slot strip byte offsets (wave-uniform); slots past the wave's range
  // repeat the last strips and are not stored
  int offA[T], offB[T];
  {
    int a, b;
    pair_tiles(min(tb, ntiles - 1), ns, 1, t0s, &a, &b);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      offA[t] = a * (32 * kG3Stride);
      offB[t] = b * (32 * kG3Stride);
      const bool wrap = b + 1 >= ns;
      const int an = wrap ? min(a + 1, ns - 1) : a;
      b = wrap ? (an > t0s ? an : t0s) : b + 1;
      a = an;
    }
  }

  f32x16 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = (f32x16){};

  const rsrc_t rs = make_rsrc(S, (uint32_t)((size_t)N * K * 4));
  const int sub = tid & 3, rb = tid >> 2;
  constexpr int kRowsPerPass = W * kWave / 4;  // 64 (W = 4) / 128 (W = 8)
  constexpr int kPasses = kG3Rows / kRowsPerPass;     // 8
  u32x4 pf[kPasses];
  auto gload1 = [&](int i, int c) {
    pf[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((rb + kRowsPerPass * i) * K + 4 * sub) * 4,
                                                  __builtin_amdgcn_readfirstlane(c * 64), 0);
  };
  auto stage1 = [&](unsigned char* buf, int i, int c) {
    const bool kv = 16 * c + 4 * sub < K;
    const u32x4 w = kv ? pf[i] : (u32x4){0u, 0u, 0u, 0u};
    if constexpr (X3)
      g3_stage(buf, rb + kRowsPerPass * i, sub, w, sc);
    else
      *reinterpret_cast<u32x4*>(buf + (rb + kRowsPerPass * i) * kG3Stride + 16 * sub) = w;
  };
  const int lofs = r * kG3Stride + (X3 ? 16 : 32) * h;
  h8 fa[2][2], fb[2][2];
  f32x8 ga[2], gb[2];
  auto rd = [&](const unsigned char* cb, int t, int s) {
    const unsigned char* pa = cb + offA[t] + lofs;
    const unsigned char* pb = cb + offB[t] + lofs;
    if constexpr (X3) {
      fa[s][0] = *reinterpret_cast<const h8*>(pa);
      fa[s][1] = *reinterpret_cast<const h8*>(pa + 32);
      fb[s][0] = *reinterpret_cast<const h8*>(pb);
      fb[s][1] = *reinterpret_cast<const h8*>(pb + 32);
    } else {
      ga[s] = *reinterpret_cast<const f32x8*>(pa);
      gb[s] = *reinterpret_cast<const f32x8*>(pb);
    }
  };

  if (c_lo < c_hi) {
#pragma unroll
    for (int i = 0; i < kPasses; ++i) gload1(i, c_lo);
#pragma unroll
    for (int i = 0; i < kPasses; ++i) {
      stage1(lds5, i, c_lo);
      gload1(i, c_lo + 1);
    }
  }
  lds_barrier();
  // chunk c: MFMAs on buf[(c - c_lo) & 1]; stage chunk c + 1 (in pf) into
  // the other buffer and refill pf with chunk c + 2.  Past the split's last
  // chunk the stage and loads run on (ignored) neighbouring data: the body
  // stays branch-free.
  for (int c = c_lo; c < c_hi; ++c) {
    const int odd = (c - c_lo) & 1;
    const unsigned char* cb = lds5 + odd * kG3Buf;
    unsigned char* nb = lds5 + (odd ^ 1) * kG3Buf;
    rd(cb, 0, 0);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (t + 1 < T) rd(cb, t + 1, (t + 1) & 1);
      if constexpr (X3) {
        acc[t] = mfma_x3(fa[t & 1][0], fa[t & 1][1], fb[t & 1][0], fb[t & 1][1], acc[t]);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(ga[t & 1][q], gb[t & 1][q], acc[t], 0, 0, 0);
      }
      if (t < kPasses) {
        stage1(nb, t, c + 1);
        gload1(t, c + 2);
      }
    }
#pragma unroll
    for (int i = T; i < kPasses; ++i) {
      stage1(nb, i, c + 1);
      gload1(i, c + 2);
    }
    lds_barrier();
  }

  const float unscale = 1.0f / (sc * sc);
#pragma unroll
  for (int t = 0; t < T; ++t) {
    if (t < nt) {
      float* out = part + ((size_t)split * ntiles + tb + t) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
        out[row * 32 + r] = acc[t][q] * unscale;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// a9 combine: per row i (one block): rowloss_i, dA row, M row.
//   loss = sum_ij A_ij (G_ii + G_jj - 2 G_ij) / 2 ; dA_ij = (G_ii+G_jj)/2 - G_ij
//   M = diag(r + c) - (A + A^T)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void surrogate_combine_kernel(const float* __restrict__ A,
                                                               const float* __restrict__ G, int N,
                                                               float* __restrict__ dA,
                                                               float* __restrict__ M,
                                                               double* __restrict__ rowloss,
                                                               _Float16* __restrict__ M16 = nullptr,
                                                               int ldm = 0, float sm = 1.0f) {
  __shared__ double sh[256];
  const int i = blockIdx.x;
  const float gii = G[(size_t)i * N + i];
  double l = 0.0, rs = 0.0, cs = 0.0;
  for (int j = threadIdx.x; j < N; j += 256) {
    const float a = A[(size_t)i * N + j];
    const float at = A[(size_t)j * N + i];
    const float gjj = G[(size_t)j * N + j];
    const float gij = G[(size_t)i * N + j];
    l += (double)a * ((double)gii + (double)gjj - 2.0 * (double)gij);
    rs += a;
    cs += at;
    if (dA) dA[(size_t)i * N + j] = 0.5f * (gii + gjj) - gij;
  }
  const double L = block_sum_256(l, sh);
  const double rc = block_sum_256(rs, sh) + block_sum_256(cs, sh);
  if (threadIdx.x == 0) rowloss[i] = 0.5 * L;
  if (M) {
    for (int j = threadIdx.x; j < N; j += 256) {
      const float a = A[(size_t)i * N + j] + A[(size_t)j * N + i];
      const float m = (i == j ? (float)rc : 0.0f) - a;
      M[(size_t)i * N + j] = m;
      if (M16) {  // the pre-split copy (split_x3_group layout, zero past N)
        const float v = m * sm;
        const _Float16 hi = (_Float16)v;
        _Float16* g = M16 + ((size_t)i * (ldm / 4) + (j >> 2)) * 8 + (j & 3);
        g[0] = hi;
        g[4] = (_Float16)(v - (float)hi);
      }
    }
    if (M16)
      for (int j = N + threadIdx.x; j < ldm; j += 256) {
        _Float16* g = M16 + ((size_t)i * (ldm / 4) + (j >> 2)) * 8 + (j & 3);
        g[0] = (_Float16)0.0f;
        g[4] = (_Float16)0.0f;
      }
  }
}

// G[i][j] = G[j][i] for i < row0 <= j: after a site-sharded all-reduce of
// the rows [row0, N) only, the leaf rows' ancestor columns take the reduced
// values (the leaf x leaf block [0, row0)^2 is a cached global constant)
__global__ __launch_bounds__(256) void gram_mirror_kernel(float* __restrict__ G, int N, int row0) {
  const int64_t n = (int64_t)row0 * (N - row0);
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int i = (int)(t / (N - row0)), j = row0 + (int)(t % (N - row0));
    G[(size_t)i * N + j] = G[(size_t)j * N + i];
  }
}

// Device step state of a graph-capturable optimisation loop
// (trex_step_advance): the 1-based step count and what the step's kernels
// derive from it -- Adam's bias corrections and the annealing schedule's
// temperature of this step and the next -- so a captured step replays with
// the right values (the reference's lax.fori_loop / scan carry,
// src/trex/evals/benchmark.py:167-200).  A null state pointer: host values.
struct StepState {
  int count;
  float bc1, bc2, T, Tn;
  float pad[3];
};
static_assert(sizeof(StepState) == 32, "step state layout");

__device__ __forceinline__ void softmax4(const float (&x)[4], float T, float (&o)[4]) {
  const float a = x[0] * T, b = x[1] * T, c = x[2] * T, d = x[3] * T;
  const float m = fmaxf(fmaxf(a, b), fmaxf(c, d));
  const float ea = expf(a - m), eb = expf(b - m), ec = expf(c - m), ed = expf(d - m);
  const float inv = 1.0f / (((ea + eb) + ec) + ed);
  o[0] = ea * inv; o[1] = eb * inv; o[2] = ec * inv; o[3] = ed * inv;
}

// One ancestor row (Q = 4) of the fused update_seq VJP + Adam + next
// update_seq: s = softmax(T p) (bitwise the S the step's GEMMs used), g = T s
// (ds - <s, ds>), Adam on p / m / v, s = softmax(Tn p_new).
__device__ __forceinline__ void adam_seq_row4(const float (&gv)[4], float (&pv)[4], float (&mv)[4],
                                              float (&vv)[4], float T, float Tn, float lr,
                                              float b1, float b2, float eps, float bc1, float bc2,
                                              float (&sv)[4]) {
  softmax4(pv, T, sv);
  float dot = sv[0] * gv[0];
#pragma unroll
  for (int q = 1; q < 4; ++q) dot = fmaf(sv[q], gv[q], dot);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float gt = T * sv[q] * (gv[q] - dot);
    const float m = (1.0f - b1) * gt + b1 * mv[q];
    const float v = (1.0f - b2) * (gt * gt) + b2 * vv[q];
    mv[q] = m;
    vv[q] = v;
    pv[q] = pv[q] + (-lr) * ((m / bc1) / (sqrtf(v / bc2) + eps));
  }
  softmax4(pv, Tn, sv);
}

// b^n by squaring in IEEE double: the host entry points and
// trex_step_advance compute the same bits (no pow() implementations to
// disagree, no contraction under -ffp-contract=off)
__host__ __device__ inline double ipow_d(double b, int n) {
  double r = 1.0;
  while (n > 0) {
    if (n & 1) r = r * b;
    b = b * b;
    n >>= 1;
  }
  return r;
}
__host__ __device__ inline float bias_corr(float b, int count) {
  return (float)(1.0 - ipow_d((double)b, count));
}

__global__ void step_advance_kernel(StepState* __restrict__ st, float b1, float b2,
                                    const float* __restrict__ temps, int64_t n_temps) {
  const int k = st->count + 1;
  st->count = k;
  st->bc1 = bias_corr(b1, k);
  st->bc2 = bias_corr(b2, k);
  if (temps && n_temps > 0) {
    st->T = temps[(int64_t)k - 1 < n_temps ? k - 1 : n_temps - 1];
    st->Tn = temps[(int64_t)k < n_temps ? k : n_temps - 1];
  }
}

// The whole surrogate for small trees (N <= 64, N K <= 4096: the NK eval
// shape is 63 x 30) in one workgroup: S, G = S S^T and M in LDS, G by
// fp32 fmaf over k in order (i <= j computed, mirrored: exactly symmetric),
// the combine's rows in fp64 (thread i sums row i over j in order), the
// loss summed over rows in order by thread 0, dS = M S.  One launch where
// the general path takes five (Gram, its reduce, combine, row sum, MF).
constexpr int kSurSmallN = 64;
constexpr int kSurSmallNK = 4096;
__global__ __launch_bounds__(1024) void surrogate_small_kernel(const float* __restrict__ S,
                                                              const float* __restrict__ A, int N,
                                                              int K, float* __restrict__ loss,
                                                              float* __restrict__ dS,
                                                              float* __restrict__ dA,
                                                              float* __restrict__ G_out) {
  constexpr int T = 1024;
  __shared__ float sS[kSurSmallNK];
  __shared__ float sG[kSurSmallN * kSurSmallN];
  __shared__ float sM[kSurSmallN * kSurSmallN];
  __shared__ float sA[kSurSmallN * kSurSmallN];
  __shared__ double part[3][kSurSmallN * 4];  // row loss, row sum, column sum partials
  __shared__ double rl[kSurSmallN];
  const int tid = threadIdx.x;
  // every operand into LDS first, all loads in flight together; each sum
  // below runs four independent partial chains combined in a fixed order (a
  // serial chain of LDS reads per entry left the block latency-bound)
  for (int e = tid; e < N * K; e += T) sS[e] = S[e];
  for (int e = tid; e < N * N; e += T) sA[e] = A[e];
  __syncthreads();
  auto dot4 = [](const float* x, int sx, const float* y, int sy, int n) {
    float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;
    int t = 0;
    for (; t + 3 < n; t += 4) {
      c0 = fmaf(x[t * sx], y[t * sy], c0);
      c1 = fmaf(x[(t + 1) * sx], y[(t + 1) * sy], c1);
      c2 = fmaf(x[(t + 2) * sx], y[(t + 2) * sy], c2);
      c3 = fmaf(x[(t + 3) * sx], y[(t + 3) * sy], c3);
    }
    for (; t < n; ++t) c0 = fmaf(x[t * sx], y[t * sy], c0);
    return (c0 + c1) + (c2 + c3);
  };
  for (int e = tid; e < N * N; e += T) {
    const int i = e / N, j = e - i * N;
    if (i > j) continue;
    const float g = dot4(sS + i * K, 1, sS + j * K, 1, K);
    sG[i * N + j] = g;
    sG[j * N + i] = g;
  }
  __syncthreads();
  // combine: row i over 4 threads (j = q, q + 4, ...), fp64 partials
  if (tid < 4 * N) {
    const int i = tid >> 2, q = tid & 3;
    const float gii = sG[i * N + i];
    double l = 0.0, rs = 0.0, cs = 0.0;
    for (int j = q; j < N; j += 4) {
      const float a = sA[i * N + j];
      const float at = sA[j * N + i];
      const float gjj = sG[j * N + j];
      const float gij = sG[i * N + j];
      l += (double)a * ((double)gii + (double)gjj - 2.0 * (double)gij);
      rs += a;
      cs += at;
      if (dA) dA[(size_t)i * N + j] = 0.5f * (gii + gjj) - gij;
      sM[i * N + j] = -(a + at);
    }
    part[0][tid] = l;
    part[1][tid] = rs;
    part[2][tid] = cs;
  }
  if (G_out)
    for (int e = tid; e < N * N; e += T) G_out[e] = sG[e];
  __syncthreads();
  if (tid < N) {
    const int i = tid;
    const double* p0 = part[0] + 4 * i;
    const double* p1 = part[1] + 4 * i;
    const double* p2 = part[2] + 4 * i;
    rl[i] = 0.5 * (((p0[0] + p0[1]) + p0[2]) + p0[3]);
    const double rc = (((p1[0] + p1[1]) + p1[2]) + p1[3]) + (((p2[0] + p2[1]) + p2[2]) + p2[3]);
    sM[i * N + i] += (float)rc;
  }
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int i = 0; i < N; ++i) t += rl[i];
    loss[0] = (float)t;
  }
  if (dS)
    for (int e = tid; e < N * K; e += T) {
      const int n = e / K, k = e - n * K;
      dS[e] = dot4(sM + n * N, 1, sS + k, K, N);
    }
}

__global__ __launch_bounds__(256) void sum_rows_kernel(const double* __restrict__ v, int n,
                                                      float scale, float* __restrict__ out,
                                                      int accumulate,
                                                      const StepState* __restrict__ ss = nullptr) {
  __shared__ double sh[256];
  if (ss) scale = ss->T;
  double s = 0.0;
  for (int t = threadIdx.x; t < n; t += 256) s += v[t];
  s = block_sum_256(s, sh);
  if (threadIdx.x == 0) out[0] = (accumulate ? out[0] : 0.0f) + (float)(s * scale);
}

// ---------------------------------------------------------------------------
// a9 dF = M F  (M [N][N], F [N][K]) on MFMA.  Column blocks are XCD-grouped:
// the row tiles of a column block share an XCD, so each F block leaves HBM
// once.
// ---------------------------------------------------------------------------

// v2 dF = M F (the f32-MFMA path; X3 = the first f16x3 version, kept
// instantiable for A/B builds, unused since MF v3): 16 n
// per step, next step's operands requested before this
// step's 32 MFMAs (ping-pong registers, unrolled by two).  Lane (r, h)
// supplies M[row][nb + 8h + t] and F[nb + 8h + t][col]; rows / n / cols past
// the edges read a clamped address and contribute 0 (M entry zeroed).
template <bool X3>
__global__ __launch_bounds__(kWave) void mf_kernel2(const float* __restrict__ Mm,
                                                   const float* __restrict__ F, int N, int K,
                                                   int row0, int nrows, int nrowt, int ncolb,
                                                   float* __restrict__ out, float sm = 1.0f,
                                                   float sf = 1.0f) {
  const int b = blockIdx.x;
  const int xcd = b & 7, m = b >> 3;
  const int rt = m % nrowt;
  const int cb = (m / nrowt) * 8 + xcd;
  if (cb >= ncolb) return;
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const int c0 = cb * 64;
  f32x16 acc[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[u][v] = (f32x16){};
  // buffer (SRD) loads: lane part of the offset in voffset, the uniform n
  // part in soffset; rows of F past N and rows of M past N read out of
  // bounds (0); n past N within an M row is masked
  const rsrc_t rm = make_rsrc(Mm, (uint32_t)((size_t)N * N * 4));
  const rsrc_t rf = make_rsrc(F, (uint32_t)((size_t)N * K * 4));
  int mvo[2], fvo[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int row = rt * 64 + u * 32 + r;  // output row; M row row0 + row
    mvo[u] = row < nrows ? ((row0 + row) * N + 8 * h) * 4 : 0x7FFFFFF0;
    const int col = c0 + u * 32 + r;
    fvo[u] = ((8 * h) * K + (col < K ? col : K - 1)) * 4;
  }
  auto fetch = [&](int nb, float (&ma)[2][8], float (&fb)[2][8]) {
    // M[row][nb + 8h .. +8): two dwordx4 loads per row (rows are only 4-byte
    // aligned; buffer loads allow that); n past N masked to 0
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int hv = 0; hv < 2; ++hv) {
        const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rm, mvo[u], (nb + 4 * hv) * 4, 0);
        const uint32_t e[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int t = 4 * hv + q;
          ma[u][t] = nb + 8 * h + t < N ? __uint_as_float(e[q]) : 0.0f;
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
#pragma unroll
      for (int v = 0; v < 2; ++v)
        fb[v][t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rf, fvo[v], (nb + t) * K * 4, 0));
    }
  };
  auto compute = [&](int nb, float (&ma)[2][8], float (&fb)[2][8]) {
    if (nb >= N) return;
    if constexpr (X3) {
      h8 mh[2], ml[2], fh[2], fl[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) split_h8(ma[u], sm, mh[u], ml[u]);
#pragma unroll
      for (int v = 0; v < 2; ++v) split_h8(fb[v], sf, fh[v], fl[v]);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) acc[u][v] = mfma_x3(mh[u], ml[u], fh[v], fl[v], acc[u][v]);
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int v = 0; v < 2; ++v)
            acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(ma[u][t], fb[v][t], acc[u][v], 0, 0, 0);
    }
  };
  float ma0[2][8], fb0[2][8], ma1[2][8], fb1[2][8];
  fetch(0, ma0, fb0);
  for (int nb = 0; nb < N; nb += 32) {
    fetch(nb + 16, ma1, fb1);
    compute(nb, ma0, fb0);
    fetch(nb + 32, ma0, fb0);
    compute(nb + 16, ma1, fb1);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = rt * 64 + u * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
        const int col = c0 + v * 32 + r;
        if (row < nrows && col < K) out[(size_t)row * K + col] = X3 ? acc[u][v][q] * (1.0f / (sm * sf)) : acc[u][v][q];
      }
}

// M row-major LDS image stride (bytes): hi n0..31 | lo n0..31 | pad
constexpr int kMfStride = 144;

typedef __fp16 fp16x4_t __attribute__((__vector_size__(4 * sizeof(__fp16))));
// two ds_read_b64_tr_b16 (rows k .. k+3 and k+4 .. k+7 of one 16-lane
// group's block) -> the 8-half B fragment of a 32x32x16 f16 MFMA
__device__ __forceinline__ h8 tr_pair(const unsigned char* p, int four_rows) {
  typedef __attribute__((address_space(3))) fp16x4_t lds_h4;
  const fp16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_h4*)(p));
  const fp16x4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_h4*)(p + four_rows));
  const h4 x = __builtin_bit_cast(h4, a), y = __builtin_bit_cast(h4, b);
  return (h8){x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

// ---- v3 MF: out = M[row0 : row0 + nrows] F, LDS-staged, persistent --------
// A workgroup (8 waves, two per SIMD) owns TPC x 32 output columns per chunk
// and up to 256 output rows (wave w: rows 32w .. 32w + 31 x all TPC column
// tiles); persistent workgroups (one per CU) walk the column chunks
// blockIdx.x + i * gridDim.x with the load pipeline running straight across
// chunk boundaries, so one chunk's output stores overlap the next chunk's
// first loads.  n advances in stages of 32 (two 32x32x16 k-steps).  Per
// stage both operands are fetched ONCE per workgroup in full 128-B lines and
// split once into f16 hi / lo:
//   * F[n .. n+32)[chunk columns] (thread item (n, cg): F[n][4cg .. +3],
//     column groups fastest) -> ROW-major LDS planes [32 n][CW] (row stride
//     SF = CW * 2 rounded to 64 mod 256 bytes: conflict-free ds_write_b64
//     and transposed reads); a B fragment (8 n of one column) is two
//     ds_read_b64_tr_b16 per plane (gfx950's transposing LDS read: lane
//     4q+p of a 16-lane group addresses row q, columns 4p..4p+3; lane i
//     receives column i of the 4 rows);
//   * M[rows][n .. n+32) (thread t: row t / 8 + 64 i, n segment t % 8) ->
//     row-major LDS [256][144 B]; an A fragment is one ds_read_b128 per
//     plane.
// Two register sets (stages s+1, s+2 in flight), LDS double-buffered, one
// barrier per stage that waits on lgkmcnt only (__syncthreads() would drain
// the prefetch).  All offsets are in voffset: rows / n past N read out of
// bounds (0).  TPC (5 or 4) is picked per launch so column tiles divide
// evenly over the CUs (C5: 1 250 chunks of 5 tiles over 256 workgroups).
// Earlier versions (same box, tools/time_gemm.py): v2 (one wave per 64x64
// tile, operands from L2) 386 us; F staged column-major with 64-B row pieces
// per load + M fragments loaded per lane 320 us; + M staged in full lines
// 296 us; this 274 us.
// CODES (Q = 4): the n stages s < lcs (F rows 0 .. 32 lcs: exact one-hot leaf
// rows) load the rows' codes (codesR [32 lcs][L] bytes, trex_tree_leaf_codes;
// an F item = one site's 4 states = one byte) instead of F and expand them
// into the same f16 hi / lo planes (one-hot x sf is exact in f16, lo = 0):
// bitwise the same result, a quarter of the bytes for those stages
// PRE: M and F pre-split (split_x3_group layout; M rows ldm elements apart,
// zero past N): the stages copy them into LDS without the split arithmetic
template <int TPC, bool CODES, bool PRE = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void mf_kernel3(
    const float* __restrict__ Mm, const float* __restrict__ F, int N, int K, int row0, int nrows,
    int nchunks, float* __restrict__ out, float sm, float sf, const uint8_t* __restrict__ codesR,
    int lcs, int ldm) {
  constexpr int CW = TPC * 32;
  constexpr int NIT = 32 * (CW / 4);  // F (row, column group) float4 items per stage
  constexpr int IPT = (NIT + 511) / 512;
  constexpr int SF = (CW * 2 + 191) / 256 * 256 + 64;  // plane row stride (bytes)
  constexpr int FPLANE = 32 * SF;
  constexpr int FBUF = 2 * FPLANE;
  constexpr int MBUF = 256 * kMfStride;
  constexpr int BUF = FBUF + MBUF;
  extern __shared__ __attribute__((aligned(16))) unsigned char ldsm[];
  const int gx = gridDim.x;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int rbase = blockIdx.y * 256 + wave * 32;
  const rsrc_t rm = make_rsrc(Mm, (uint32_t)((size_t)N * ldm * 4));
  const rsrc_t rf = make_rsrc(F, (uint32_t)((size_t)N * K * 4));
  // CODES: item (n, cg) reads the code byte of row n, site chunk * CW / 4 + cg
  // (sites past L read the next row's bytes: columns past K, never stored)
  const int Lc = K / 4;
  const rsrc_t rc = make_rsrc(codesR, (uint32_t)(CODES ? (size_t)Lc * 32 * lcs : 0));
  int cvb[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int item = tid + 512 * j;
    cvb[j] = (item < NIT) ? (item / (CW / 4)) * Lc + item % (CW / 4) : 0x7FFF0000;
  }
  int fvb[IPT], lofs[IPT];
  bool fok[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int item = tid + 512 * j;
    fok[j] = item < NIT;
    const int n = fok[j] ? item / (CW / 4) : 0, cg = fok[j] ? item % (CW / 4) : 0;
    fvb[j] = (n * K + 4 * cg) * 4;
    lofs[j] = n * SF + 8 * cg;
  }
  // M staging: thread t covers rows t / 8 + 64 i (i < 4), n segment t % 8
  const int mseg = tid & 7, mrow = tid >> 3;
  int mvb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rg = blockIdx.y * 256 + mrow + 64 * i;
    mvb[i] = rg < nrows ? ((row0 + rg) * ldm + 4 * mseg) * 4 : -1;
  }
  const int nst = (N + 31) / 32;
  const int cnt = blockIdx.x < nchunks ? (nchunks - 1 - (int)blockIdx.x) / gx + 1 : 0;
  const int G = cnt * nst;

  f32x16 acc[TPC];
#pragma unroll
  for (int t = 0; t < TPC; ++t) acc[t] = (f32x16){};

  struct Set { u32x4 a[IPT], m[4]; int s; };
  Set r0, r1;
  int fc = blockIdx.x, fs = 0;  // load cursor (chunk, stage)
  int cc = blockIdx.x, cs = 0;  // compute cursor
  auto load = [&](Set& q) {
    if (CODES && fs < lcs) {
      const int so = fs * 32 * Lc + fc * (CW / 4);
#pragma unroll
      for (int j = 0; j < IPT; ++j)
        q.a[j].x = __builtin_amdgcn_raw_buffer_load_b8(rc, cvb[j] < 0x7FFF0000 ? cvb[j] + so : cvb[j], 0, 0);
    } else {
      const int so = (fc * CW + fs * 32 * K) * 4;
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        const int vo = fok[j] ? fvb[j] + so : 0x7FFF0000;
        q.a[j] = __builtin_amdgcn_raw_buffer_load_b128(rf, vo, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      q.m[i] = __builtin_amdgcn_raw_buffer_load_b128(rm, mvb[i] < 0 ? 0x7FFF0000 : mvb[i] + fs * 128,
                                                     0, 0);
    q.s = fs;
    if (++fs == nst) { fs = 0; fc += gx; }
  };
  const uint32_t hb = (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)sf);  // one-hot 1 x sf
  auto stage = [&](unsigned char* buf, const Set& q) {
    if (CODES && q.s < lcs) {
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        if (!fok[j]) continue;
        const uint32_t code = q.a[j].x & 0xFFu;
        *reinterpret_cast<uint2*>(buf + lofs[j]) =
            uint2{(code == 0 ? hb : 0u) | ((code == 1 ? hb : 0u) << 16),
                  (code == 2 ? hb : 0u) | ((code == 3 ? hb : 0u) << 16)};
        // the lo plane (zero) is not staged: compute skips its products
#ifdef TREX_NO_LZ
        *reinterpret_cast<uint2*>(buf + FPLANE + lofs[j]) = uint2{0u, 0u};
#endif
      }
    }
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      if (!fok[j] || (CODES && q.s < lcs)) continue;
      if constexpr (PRE) {
        *reinterpret_cast<uint2*>(buf + lofs[j]) = uint2{q.a[j].x, q.a[j].y};
        *reinterpret_cast<uint2*>(buf + FPLANE + lofs[j]) = uint2{q.a[j].z, q.a[j].w};
        continue;
      }
      const uint32_t e[4] = {q.a[j].x, q.a[j].y, q.a[j].z, q.a[j].w};
      h4 hi, lo;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float v = __uint_as_float(e[c]) * sf;
        hi[c] = (_Float16)v;
        lo[c] = (_Float16)(v - (float)hi[c]);
      }
      *reinterpret_cast<h4*>(buf + lofs[j]) = hi;
      *reinterpret_cast<h4*>(buf + FPLANE + lofs[j]) = lo;
    }
    unsigned char* mb = buf + FBUF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (PRE) {
        unsigned char* rowp = mb + (mrow + 64 * i) * kMfStride + 8 * mseg;
        *reinterpret_cast<uint2*>(rowp) = uint2{q.m[i].x, q.m[i].y};
        *reinterpret_cast<uint2*>(rowp + 64) = uint2{q.m[i].z, q.m[i].w};
        continue;
      }
      const uint32_t e[4] = {q.m[i].x, q.m[i].y, q.m[i].z, q.m[i].w};
      h4 hi, lo;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float v = (q.s * 32 + 4 * mseg + c < N) ? __uint_as_float(e[c]) * sm : 0.0f;
        hi[c] = (_Float16)v;
        lo[c] = (_Float16)(v - (float)hi[c]);
      }
      unsigned char* row = mb + (mrow + 64 * i) * kMfStride + 8 * mseg;
      *reinterpret_cast<h4*>(row) = hi;
      *reinterpret_cast<h4*>(row + 64) = lo;
    }
  };
  // transposed-read lane address: group g = lane / 16, lane 4q + p of it
  // addresses row 8 (g / 2) + q, columns 16 (g % 2) + 4p .. + 3
  const int trk = 8 * (lane >> 5) + ((lane & 15) >> 2);
  const int trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const float unscale = 1.0f / (sm * sf);
  auto compute = [&](const unsigned char* buf) {
    const unsigned char* pa = buf + FBUF + (wave * 32 + r) * kMfStride + 16 * h;
    // leaf-code stages: F's lo plane is zero (one-hot x sf is exact in f16),
    // so its ah x bl products -- exact zeros -- are skipped (bitwise)
#ifdef TREX_NO_LZ
    const bool zlo = false;  // A/B: every product computed
#else
    const bool zlo = CODES && cs < lcs;
#endif
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const h8 ah = *reinterpret_cast<const h8*>(pa + kk * 32);
      const h8 al = *reinterpret_cast<const h8*>(pa + kk * 32 + 64);
#pragma unroll
      for (int t = 0; t < TPC; ++t) {
        const int o1 = (kk * 16 + trk) * SF + (t * 32 + trc) * 2;
        const h8 bh = tr_pair(buf + o1, 4 * SF);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[t], 0, 0, 0);
        if (!zlo) {
          const h8 bl = tr_pair(buf + FPLANE + o1, 4 * SF);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[t], 0, 0, 0);
        }
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[t], 0, 0, 0);
      }
    }
    if (++cs == nst) {  // chunk done: store its tile, restart the accumulators
      if (rbase < nrows) {
#pragma unroll
        for (int t = 0; t < TPC; ++t) {
          const int col = cc * CW + t * 32 + r;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int row = rbase + (q & 3) + 8 * (q >> 2) + 4 * h;
            if (row < nrows && col < K) out[(size_t)row * K + col] = acc[t][q] * unscale;
          }
        }
      }
#pragma unroll
      for (int t = 0; t < TPC; ++t) acc[t] = (f32x16){};
      cs = 0;
      cc += gx;
    }
  };

  if (G == 0) return;
  unsigned char* buf0 = ldsm;
  unsigned char* buf1 = ldsm + BUF;
  load(r0);
  load(r1);
  stage(buf0, r0);
  load(r0);
  lds_barrier();
  for (int g = 0; g < G; g += 2) {
    compute(buf0);
    if (g + 1 < G) stage(buf1, r1);
    load(r1);
    lds_barrier();
    if (g + 1 >= G) break;
    compute(buf1);
    if (g + 2 < G) stage(buf0, r0);
    load(r0);
    lds_barrier();
  }
}

// ---- v5 MF: one wave per SIMD, pipelined fragment reads --------------------
// v3's chunking, LDS images and leaf-code stages with Gram v5's structure: a
// workgroup is 4 waves (one per SIMD, accumulators in AGPRs), wave w owns
// output rows 64w .. 64w + 63 (two row tiles) x the chunk's TPC column tiles,
// so each B fragment (4 transposed reads) feeds 2 x 3 MFMAs and each A
// fragment TPC x 3.  One register set of raw operands: the stage-(s + 1)
// f16 split and the stage-(s + 2) loads ride between the stage-s MFMAs
// (one raw item after each column tile), with no branch in the stage body
// (loads past the split run on neighbouring data or out of bounds: 0, and
// stage into the buffer nobody reads next).
template <int TPC, bool CODES, bool X3>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void mf_kernel5(
    const float* __restrict__ Mm, const float* __restrict__ F, int N, int K, int row0, int nrows,
    int nchunks, float* __restrict__ out, float sm, float sf, const uint8_t* __restrict__ codesR,
    int lcs) {
  constexpr int CW = TPC * 32;
  constexpr int NIT = 32 * (CW / 4);  // F (row, column group) float4 items per stage
  constexpr int IPT = (NIT + 255) / 256;
  constexpr int SF = (CW * 2 + 191) / 256 * 256 + 64;  // plane row stride (bytes)
  constexpr int FPLANE = 32 * SF;
  // X3: f16 hi / lo planes [32 n][SF]; f32: the F slice transposed [CW][32 n]
  // (144-B columns: a lane's 8 n are two ds_read_b128, conflict-free)
  constexpr int FBUF = X3 ? 2 * FPLANE : CW * kMfStride;
  static_assert(X3 || !CODES, "leaf codes ride on the x3 path only");
  constexpr int MBUF = 256 * kMfStride;
  constexpr int BUF = FBUF + MBUF;
  constexpr int MPT = 8;  // M float4 items per thread: rows tid / 8 + 32 i
  constexpr int NRAW = IPT + MPT;
  extern __shared__ __attribute__((aligned(16))) unsigned char ldsm5[];
  const int gx = gridDim.x;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int rbase = blockIdx.y * 256 + wave * 64;
  // M rows row0 .. row0 + nrows - 1 only: rows past them read out of bounds (0)
  const rsrc_t rm = make_rsrc(Mm + (size_t)row0 * N, (uint32_t)((size_t)nrows * N * 4));
  // output rows 0 .. nrows - 1: stores past them are dropped by the bounds check
  const rsrc_t ro = make_rsrc(out, (uint32_t)((size_t)nrows * K * 4));
  const rsrc_t rf = make_rsrc(F, (uint32_t)((size_t)N * K * 4));
  const int Lc = K / 4;
  const rsrc_t rc = make_rsrc(codesR, (uint32_t)(CODES ? (size_t)Lc * 32 * lcs : 0));
  static_assert(NIT % 256 == 0, "F items tile the workgroup exactly");
  int fvb[IPT], lofs[IPT], cvb[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int item = tid + 256 * j;
    const int n = item / (CW / 4), cg = item % (CW / 4);
    fvb[j] = (n * K + 4 * cg) * 4;
    lofs[j] = X3 ? n * SF + 8 * cg : 4 * cg * kMfStride + 4 * n;
    cvb[j] = n * Lc + cg;
  }
  const int mseg = tid & 7, mrow = tid >> 3;
  const int mvb = ((blockIdx.y * 256 + mrow) * N + 4 * mseg) * 4;  // + i * 32 rows
  const int nst = (N + 31) / 32;
  const int cnt = blockIdx.x < nchunks ? (nchunks - 1 - (int)blockIdx.x) / gx + 1 : 0;
  const int G = cnt * nst;
  if (G == 0) return;

  f32x16 acc[2][TPC];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int t = 0; t < TPC; ++t) acc[u][t] = (f32x16){};

  u32x4 raw[NRAW];
  uint32_t rcode[CODES ? IPT : 1];
  // raw item i of (chunk fc, stage fs): F items first, then M.  CODES: a
  // leaf-code stage's F items come from the code bytes instead -- both loads
  // are issued, the unused one out of bounds (no memory request), so the
  // stage body has no branch
  auto load1 = [&](int i, int fc, int fs) {
    if (i < IPT) {
      const bool code = CODES && fs < lcs;
      const int so = __builtin_amdgcn_readfirstlane(code ? 0x7FFF0000 : (fc * CW + fs * 32 * K) * 4);
      raw[i] = __builtin_amdgcn_raw_buffer_load_b128(rf, fvb[i], so, 0);
      if (CODES) {
        const int sc = __builtin_amdgcn_readfirstlane(code ? fs * 32 * Lc + fc * (CW / 4) : 0x7FFF0000);
        rcode[i] = __builtin_amdgcn_raw_buffer_load_b8(rc, cvb[i], sc, 0);
      }
    } else {
      raw[i] = __builtin_amdgcn_raw_buffer_load_b128(
          rm, mvb, __builtin_amdgcn_readfirstlane(fs * 128 + (i - IPT) * 32 * N * 4), 0);
    }
  };
  // one-hot x sf is exact in f16 (sf a power of two <= 2^14): a code item's
  // hi plane is the one-hot pattern and its lo plane 0, as the f32 rows give
  auto stage1 = [&](unsigned char* buf, int i, int fs) {
    if (i < IPT) {
      float e[4] = {__uint_as_float(raw[i].x), __uint_as_float(raw[i].y),
                    __uint_as_float(raw[i].z), __uint_as_float(raw[i].w)};
      if (CODES) {
        const bool code = fs < lcs;
        const uint32_t cv = rcode[i] & 0xFFu;
#pragma unroll
        for (int c = 0; c < 4; ++c) e[c] = code ? (cv == (uint32_t)c ? 1.0f : 0.0f) : e[c];
      }
      if constexpr (!X3) {
#pragma unroll
        for (int c = 0; c < 4; ++c) *reinterpret_cast<float*>(buf + lofs[i] + c * kMfStride) = e[c];
        return;
      }
      h4 hi, lo;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float v = e[c] * sf;
        hi[c] = (_Float16)v;
        lo[c] = (_Float16)(v - (float)hi[c]);
      }
      *reinterpret_cast<h4*>(buf + lofs[i]) = hi;
      *reinterpret_cast<h4*>(buf + FPLANE + lofs[i]) = lo;
    } else {
      const int mi = i - IPT;
      const uint32_t e[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
      if constexpr (!X3) {
        float4 v;
        v.x = (fs * 32 + 4 * mseg < N) ? __uint_as_float(e[0]) : 0.0f;
        v.y = (fs * 32 + 4 * mseg + 1 < N) ? __uint_as_float(e[1]) : 0.0f;
        v.z = (fs * 32 + 4 * mseg + 2 < N) ? __uint_as_float(e[2]) : 0.0f;
        v.w = (fs * 32 + 4 * mseg + 3 < N) ? __uint_as_float(e[3]) : 0.0f;
        *reinterpret_cast<float4*>(buf + FBUF + (mrow + 32 * mi) * kMfStride + 16 * mseg) = v;
        return;
      }
      h4 hi, lo;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float v = (fs * 32 + 4 * mseg + c < N) ? __uint_as_float(e[c]) * sm : 0.0f;
        hi[c] = (_Float16)v;
        lo[c] = (_Float16)(v - (float)hi[c]);
      }
      unsigned char* row = buf + FBUF + (mrow + 32 * mi) * kMfStride + 8 * mseg;
      *reinterpret_cast<h4*>(row) = hi;
      *reinterpret_cast<h4*>(row + 64) = lo;
    }
  };
  const int trk = 8 * (lane >> 5) + ((lane & 15) >> 2);
  const int trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const float unscale = X3 ? 1.0f / (sm * sf) : 1.0f;

  // cursors: compute (cc, cs); staged stage = compute + 1; loaded = + 2
  int cc = blockIdx.x, cs = 0;
  int sc_ = cs + 1, scc = cc;  // staged-stage cursor
  if (sc_ == nst) { sc_ = 0; scc += gx; }
  int lc = scc, ls = sc_ + 1;  // load cursor
  if (ls == nst) { ls = 0; lc += gx; }
  unsigned char* buf0 = ldsm5;
  unsigned char* buf1 = ldsm5 + BUF;
#pragma unroll
  for (int i = 0; i < NRAW; ++i) load1(i, cc, cs);
#pragma unroll
  for (int i = 0; i < NRAW; ++i) {
    stage1(buf0, i, cs);
    load1(i, scc, sc_);
  }
  lds_barrier();
  for (int g = 0; g < G; ++g) {
    const unsigned char* cb = (g & 1) ? buf1 : buf0;
    unsigned char* nb = (g & 1) ? buf0 : buf1;
    const unsigned char* pa = cb + FBUF + (wave * 64 + r) * kMfStride + 16 * h;
    int item = 0;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      h8 ah[2], al[2];
      f32x8 fa[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if constexpr (X3) {
          ah[u] = *reinterpret_cast<const h8*>(pa + u * 32 * kMfStride + kk * 32);
          al[u] = *reinterpret_cast<const h8*>(pa + u * 32 * kMfStride + kk * 32 + 64);
        } else {  // n = 16 kk + 8 h .. + 7 (pa carries 16 h bytes: one more 16 h)
          fa[u] = *reinterpret_cast<const f32x8*>(pa + u * 32 * kMfStride + kk * 64 + 16 * h);
        }
      }
#pragma unroll
      for (int t = 0; t < TPC; ++t) {
        if constexpr (X3) {
          const int o1 = (kk * 16 + trk) * SF + (t * 32 + trc) * 2;
          const h8 bh = tr_pair(cb + o1, 4 * SF);
          const h8 bl = tr_pair(cb + FPLANE + o1, 4 * SF);
#pragma unroll
          for (int u = 0; u < 2; ++u) acc[u][t] = mfma_x3(ah[u], al[u], bh, bl, acc[u][t]);
        } else {
          // MFMA q covers n = 16 kk + q and 16 kk + 8 + q on the two lane halves
          const f32x8 fb = *reinterpret_cast<const f32x8*>(cb + (t * 32 + r) * kMfStride + kk * 64 + 32 * h);
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int q = 0; q < 8; ++q)
              acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[u][q], fb[q], acc[u][t], 0, 0, 0);
        }
        // one raw item per column tile: staged for stage + 1, refilled for + 2
        if (item < NRAW) {
          stage1(nb, item, sc_);
          load1(item, lc, ls);
          ++item;
        }
      }
    }
#pragma unroll
    for (int i = 2 * TPC; i < NRAW; ++i) {
      stage1(nb, i, sc_);
      load1(i, lc, ls);
    }
    if (++ls == nst) { ls = 0; lc += gx; }
    if (++sc_ == nst) { sc_ = 0; scc += gx; }
    if (++cs == nst) {  // chunk done: store its tiles, restart the accumulators
      // branch-free: columns past K (a ragged last tile) get an out-of-
      // bounds offset, rows past nrows fall outside the store resource
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int t = 0; t < TPC; ++t) {
          const int col = cc * CW + t * 32 + r;
          const int row = rbase + u * 32 + 4 * h;
          const int vo = (col < K && row < nrows) ? (row * K + col) * 4 : 0x7FFFFFF0;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int dr = (q & 3) + 8 * (q >> 2);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[u][t][q] * unscale), ro,
                                                  vo, __builtin_amdgcn_readfirstlane(dr * K * 4), 0);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int t = 0; t < TPC; ++t) acc[u][t] = (f32x16){};
      cs = 0;
      cc += gx;
    }
    lds_barrier();
  }
}

int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

// ---------------------------------------------------------------------------
// a10 W = S C per (node, site):  ckind 0: W = S; 1: W = S * c (vector);
//     2: W = S @ C (matrix, w_j = sum_q s_q C[q][j])
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void weight_seq_kernel(const float* __restrict__ S, int64_t rows,
                                                        int Q, const float* __restrict__ C,
                                                        int ckind, float* __restrict__ W) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    const float* s = S + r * Q;
    for (int j = 0; j < Q; ++j) {
      float w;
      if (ckind == 0) {
        w = s[j];
      } else if (ckind == 1) {
        w = s[j] * C[j];
      } else {
        w = 0.0f;
        for (int q = 0; q < Q; ++q) w = fmaf(s[q], C[q * Q + j], w);
      }
      W[r * Q + j] = w;
    }
  }
}

// soft-cost combine: loss_i = sum_j A_ij (E_i + E_j - 2 G_ij) / 2, E = diag(G)
// (E_i = sum S_i * W_i = <S_i, W_i>, tree.py:255)
__global__ __launch_bounds__(256) void soft_combine_kernel(const float* __restrict__ A,
                                                          const float* __restrict__ G, int N,
                                                          double* __restrict__ rowloss) {
  __shared__ double sh[256];
  const int i = blockIdx.x;
  const double ei = G[(size_t)i * N + i];
  double l = 0.0;
  for (int j = threadIdx.x; j < N; j += 256)
    l += (double)A[(size_t)i * N + j] *
         (ei + (double)G[(size_t)j * N + j] - 2.0 * (double)G[(size_t)i * N + j]);
  l = block_sum_256(l, sh);
  if (threadIdx.x == 0) rowloss[i] = 0.5 * l;
}

// ---------------------------------------------------------------------------
// a13 constraint: scale * sum_cols (sum_{i<N-1} A[i][c] - 2)^2, c in last n_anc
//   grad (x gscale, accumulated into dA): 2 scale (colsum - 2)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void constraint_kernel(const float* __restrict__ A, int N,
                                                        float scale, float gscale,
                                                        double* __restrict__ colloss,
                                                        float* __restrict__ dA,
                                                        const StepState* __restrict__ ss) {
  __shared__ double sh[256];
  if (ss) gscale = ss->T;
  const int n_anc = (N - 1) / 2;
  const int c = N - n_anc + blockIdx.x;
  double s = 0.0;
  for (int i = threadIdx.x; i < N - 1; i += 256) s += A[(size_t)i * N + c];
  s = block_sum_256(s, sh);
  const double dev = s - 2.0;
  if (threadIdx.x == 0) colloss[blockIdx.x] = (double)scale * dev * dev;
  if (dA) {
    const float g = (float)(2.0 * scale * dev) * gscale;
    for (int i = threadIdx.x; i < N - 1; i += 256) dA[(size_t)i * N + c] += g;
  }
}

// ---------------------------------------------------------------------------
// a8 compute_cost: seq = argmax_q S, parent = argmax_j A (first index), sum
//   subst[seq[parent][l]][seq[i][l]] over i < N-1, l.  One block per node i.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void compute_cost_kernel(const float* __restrict__ S,
                                                          const float* __restrict__ A,
                                                          const float* __restrict__ subst, int N,
                                                          int L, int Q,
                                                          double* __restrict__ rowcost) {
  __shared__ double sh[256];
  __shared__ float bv[256];
  __shared__ int bi[256];
  const int i = blockIdx.x;
  // parent = first argmax of row i
  float best = -INFINITY;
  int arg = 0x7FFFFFFF;
  for (int j = threadIdx.x; j < N; j += 256) {
    const float v = A[(size_t)i * N + j];
    if (v > best || (v == best && j < arg)) { best = v; arg = j; }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = arg;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      const float v = bv[threadIdx.x + w];
      const int k = bi[threadIdx.x + w];
      if (v > bv[threadIdx.x] || (v == bv[threadIdx.x] && k < bi[threadIdx.x])) {
        bv[threadIdx.x] = v;
        bi[threadIdx.x] = k;
      }
    }
    __syncthreads();
  }
  const int p = bi[0] == 0x7FFFFFFF ? 0 : bi[0];
  double s = 0.0;
  for (int l = threadIdx.x; l < L; l += 256) {
    const float* si = S + ((size_t)i * L + l) * Q;
    const float* sp = S + ((size_t)p * L + l) * Q;
    int a = 0, c = 0;
    float va = si[0], vc = sp[0];
    for (int q = 1; q < Q; ++q) {
      if (si[q] > va) { va = si[q]; a = q; }
      if (sp[q] > vc) { vc = sp[q]; c = q; }
    }
    s += subst[c * Q + a];
  }
  s = block_sum_256(s, sh);
  if (threadIdx.x == 0) rowcost[i] = s;
}

// ---------------------------------------------------------------------------
// a14 optax adam (b1, b2, eps; eps_root = 0) with optional global-norm clip
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sq_norm_kernel(const float* __restrict__ g, int64_t n,
                                                     double* __restrict__ part) {
  __shared__ double sh[256];
  double s = 0.0;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256)
    s += (double)g[t] * (double)g[t];
  s = block_sum_256(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p,
                                                  const float* __restrict__ g,
                                                  float* __restrict__ mu, float* __restrict__ nu,
                                                  int64_t n, float lr, float b1, float b2,
                                                  float eps, float bc1, float bc2,
                                                  const double* __restrict__ sqnorm,
                                                  int nparts, float clip,
                                                  const StepState* __restrict__ ss) {
  if (ss) {
    bc1 = ss->bc1;
    bc2 = ss->bc2;
  }
  float scale = 1.0f;
  if (sqnorm) {
    double s = 0.0;
    for (int k = 0; k < nparts; ++k) s += sqnorm[k];  // same fixed order in every thread
    const float norm = (float)sqrt(s);
    if (!(norm < clip)) scale = clip / norm;
  }
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const float gt = (scale == 1.0f) ? g[t] : (g[t] / (clip / scale)) * clip;
    const float m = (1.0f - b1) * gt + b1 * mu[t];
    const float v = (1.0f - b2) * (gt * gt) + b2 * nu[t];
    mu[t] = m;
    nu[t] = v;
    const float mh = m / bc1;
    const float vh = v / bc2;
    p[t] = p[t] + (-lr) * (mh / (sqrtf(vh) + eps));
  }
}

// update_tree's VJP (update_tree_bwd_kernel's arithmetic) with the
// tree_params' Adam step (adam_kernel's, no clip) applied in the same pass:
// one block per row, the gradient optionally written out as well
__global__ __launch_bounds__(256) void update_tree_bwd_adam_kernel(
    const float* __restrict__ A, const float* __restrict__ dA, const float* __restrict__ gates,
    int N, int n_anc, float T, float* __restrict__ dtheta, float* __restrict__ p,
    float* __restrict__ mu, float* __restrict__ nu, float lr, float b1, float b2, float eps,
    float bc1, float bc2, const StepState* __restrict__ ss) {
  __shared__ double sh[256];
  if (ss) {
    bc1 = ss->bc1;
    bc2 = ss->bc2;
  }
  const int i = blockIdx.x;  // rows 0..N-2
  const int nl = N - n_anc;
  double dot = 0.0;
  for (int j = threadIdx.x; j < N; j += 256)
    dot += (double)A[(size_t)i * N + j] * (double)dA[(size_t)i * N + j];
  const float d = (float)block_sum_256(dot, sh);
  for (int ja = threadIdx.x; ja < n_anc; ja += 256) {
    const int j = nl + ja;
    const bool valid = (i < nl) || (ja > i - nl);
    float g = 0.0f;
    if (valid) {
      const float a = A[(size_t)i * N + j];
      g = a * (dA[(size_t)i * N + j] - d) / T;
      if (gates) g *= gates[(size_t)i * n_anc + ja];
    }
    const size_t t = (size_t)i * n_anc + ja;
    if (dtheta) dtheta[t] = g;
    const float m = (1.0f - b1) * g + b1 * mu[t];
    const float v = (1.0f - b2) * (g * g) + b2 * nu[t];
    mu[t] = m;
    nu[t] = v;
    const float mh = m / bc1;
    const float vh = v / bc2;
    p[t] = p[t] + (-lr) * (mh / (sqrtf(vh) + eps));
  }
}

// loss = rows (x 1) then + cols x gscale: the two sum_rows_kernel launches of
// trex_tree_surrogate_combine + trex_tree_constraint in one, same arithmetic
__global__ __launch_bounds__(256) void sum_rows2_kernel(const double* __restrict__ v1, int n1,
                                                       const double* __restrict__ v2, int n2,
                                                       float scale2, float* __restrict__ out,
                                                       const StepState* __restrict__ ss) {
  __shared__ double sh[256];
  if (ss) scale2 = ss->T;
  double s = 0.0;
  for (int t = threadIdx.x; t < n1; t += 256) s += v1[t];
  s = block_sum_256(s, sh);
  double s2 = 0.0;
  for (int t = threadIdx.x; t < n2; t += 256) s2 += v2[t];
  s2 = block_sum_256(s2, sh);
  if (threadIdx.x == 0) {
    const float first = 0.0f + (float)(s * 1.0f);
    out[0] = first + (float)(s2 * scale2);
  }
}

// optax transformations of src/trex/evals/benchmark.py:41-72
// (create_optimizer), optionally after clip_by_global_norm:
//   kind 0 adam(lr, b1, b2, eps)        s1 = mu, s2 = nu (bias-corrected)
//   kind 1 adamw(lr, ..., wd)           adam + wd * p, then * -lr
//   kind 2 sgd(lr, momentum = b1)       s1 = trace: t = g + b1 t
//   kind 3 rmsprop(lr, decay = b2, eps) s2 = nu = b2 nu + (1 - b2) g^2,
//                                       update g / sqrt(nu + eps)
// (optax 0.2.6 defaults: eps_root 0, nesterov off, rmsprop eps inside sqrt,
// initial_scale 0, not centred).
__global__ __launch_bounds__(256) void optax_kernel(int kind, float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ s1,
                                                   float* __restrict__ s2, int64_t n, float lr,
                                                   float b1, float b2, float eps, float wd,
                                                   float bc1, float bc2,
                                                   const double* __restrict__ sqnorm,
                                                   int nparts, float clip,
                                                   const StepState* __restrict__ ss) {
  if (ss) {
    bc1 = ss->bc1;
    bc2 = ss->bc2;
  }
  float scale = 1.0f;
  if (sqnorm) {
    double sum = 0.0;
    for (int k = 0; k < nparts; ++k) sum += sqnorm[k];  // same fixed order in every thread
    const float norm = (float)sqrt(sum);
    if (!(norm < clip)) scale = clip / norm;
  }
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const float gt = (scale == 1.0f) ? g[t] : (g[t] / (clip / scale)) * clip;
    float u;
    if (kind <= 1) {
      const float m = (1.0f - b1) * gt + b1 * s1[t];
      const float v = (1.0f - b2) * (gt * gt) + b2 * s2[t];
      s1[t] = m;
      s2[t] = v;
      u = (m / bc1) / (sqrtf(v / bc2) + eps);
      if (kind == 1) u = u + wd * p[t];
    } else if (kind == 2) {
      u = gt + b1 * s1[t];
      s1[t] = u;
    } else {
      const float v = (1.0f - b2) * (gt * gt) + b2 * s2[t];
      s2[t] = v;
      u = gt / sqrtf(v + eps);
    }
    p[t] = p[t] + (-lr) * u;
  }
}

// update_seq VJP fused into the optax Adam update of the ancestor logits
// (no clip): g = T s (ds - <s, ds>) per (ancestor, site) row of Q states,
// then the same Adam arithmetic as adam_kernel; g never touches HBM unless
// g_out is given.  Q = 4 rows move as float4.
template <int QT>
__global__ __launch_bounds__(256) void adam_seq_kernel(const float* __restrict__ s,
                                                      const float* __restrict__ ds, int64_t rows,
                                                      int Qr, float T, float* __restrict__ p,
                                                      float* __restrict__ mu,
                                                      float* __restrict__ nu, float lr, float b1,
                                                      float b2, float eps, float bc1, float bc2,
                                                      float* __restrict__ g_out) {
  const int Q = QT ? QT : Qr;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < rows; r += (int64_t)gridDim.x * 256) {
    float sv[QT ? QT : 32], gv[QT ? QT : 32];
    if constexpr (QT == 4) {
      const float4 a = reinterpret_cast<const float4*>(s)[r];
      const float4 d = reinterpret_cast<const float4*>(ds)[r];
      sv[0] = a.x; sv[1] = a.y; sv[2] = a.z; sv[3] = a.w;
      gv[0] = d.x; gv[1] = d.y; gv[2] = d.z; gv[3] = d.w;
    } else {
      for (int q = 0; q < Q; ++q) {
        sv[q] = s[r * Q + q];
        gv[q] = ds[r * Q + q];
      }
    }
    float dot = sv[0] * gv[0];
    for (int q = 1; q < Q; ++q) dot = fmaf(sv[q], gv[q], dot);
    float pv[QT ? QT : 32], mv[QT ? QT : 32], vv[QT ? QT : 32];
    if constexpr (QT == 4) {
      const float4 a = reinterpret_cast<const float4*>(p)[r];
      const float4 m = reinterpret_cast<const float4*>(mu)[r];
      const float4 v = reinterpret_cast<const float4*>(nu)[r];
      pv[0] = a.x; pv[1] = a.y; pv[2] = a.z; pv[3] = a.w;
      mv[0] = m.x; mv[1] = m.y; mv[2] = m.z; mv[3] = m.w;
      vv[0] = v.x; vv[1] = v.y; vv[2] = v.z; vv[3] = v.w;
    } else {
      for (int q = 0; q < Q; ++q) {
        pv[q] = p[r * Q + q];
        mv[q] = mu[r * Q + q];
        vv[q] = nu[r * Q + q];
      }
    }
    for (int q = 0; q < Q; ++q) {
      const float gt = T * sv[q] * (gv[q] - dot);
      gv[q] = gt;
      const float m = (1.0f - b1) * gt + b1 * mv[q];
      const float v = (1.0f - b2) * (gt * gt) + b2 * vv[q];
      mv[q] = m;
      vv[q] = v;
      pv[q] = pv[q] + (-lr) * ((m / bc1) / (sqrtf(v / bc2) + eps));
    }
    if constexpr (QT == 4) {
      reinterpret_cast<float4*>(p)[r] = make_float4(pv[0], pv[1], pv[2], pv[3]);
      reinterpret_cast<float4*>(mu)[r] = make_float4(mv[0], mv[1], mv[2], mv[3]);
      reinterpret_cast<float4*>(nu)[r] = make_float4(vv[0], vv[1], vv[2], vv[3]);
      if (g_out) reinterpret_cast<float4*>(g_out)[r] = make_float4(gv[0], gv[1], gv[2], gv[3]);
    } else {
      for (int q = 0; q < Q; ++q) {
        p[r * Q + q] = pv[q];
        mu[r * Q + q] = mv[q];
        nu[r * Q + q] = vv[q];
        if (g_out) g_out[r * Q + q] = gv[q];
      }
    }
  }
}

// One ancestor-logits step with update_seq folded in on both sides: s =
// softmax(T p) recomputed from the logits it reads anyway (the same
// arithmetic as update_seq_kernel, so bitwise the S the step's GEMMs used),
// the VJP g = T s (ds - <s, ds>), the Adam update of p / mu / nu, and the
// NEXT step's S rows softmax(Tn p_new) written to s_out: per row of Q
// logits 16 B of ds + 12 B of Adam state in, 16 B + 12 B out, no separate
// update_seq pass (which re-read p) and no read of the old S.
__device__ __forceinline__ void softmaxq(const float* x, int Q, float T, float* o) {
  float m = -INFINITY;
  for (int q = 0; q < Q; ++q) m = fmaxf(m, x[q] * T);
  float sum = 0.0f;
  for (int q = 0; q < Q; ++q) sum += expf(x[q] * T - m);
  const float inv = 1.0f / sum;
  for (int q = 0; q < Q; ++q) o[q] = expf(x[q] * T - m) * inv;
}

// any Q <= 32 (a grid-stride loop over rows)
__global__ __launch_bounds__(256) void adam_seq_update_kernel(
    const float* __restrict__ ds, int64_t rows, int Q, float T, float Tn, float* __restrict__ p,
    float* __restrict__ mu, float* __restrict__ nu, float lr, float b1, float b2, float eps,
    float bc1, float bc2, float* __restrict__ s_out, const StepState* __restrict__ ss) {
  if (ss) {
    bc1 = ss->bc1;
    bc2 = ss->bc2;
    T = ss->T;
    Tn = ss->Tn;
  }
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < rows; r += (int64_t)gridDim.x * 256) {
    float pv[32], mv[32], vv[32], gv[32], sv[32];
    for (int q = 0; q < Q; ++q) {
      pv[q] = p[r * Q + q];
      gv[q] = ds[r * Q + q];
      mv[q] = mu[r * Q + q];
      vv[q] = nu[r * Q + q];
    }
    softmaxq(pv, Q, T, sv);
    float dot = sv[0] * gv[0];
    for (int q = 1; q < Q; ++q) dot = fmaf(sv[q], gv[q], dot);
    for (int q = 0; q < Q; ++q) {
      const float gt = T * sv[q] * (gv[q] - dot);
      const float m = (1.0f - b1) * gt + b1 * mv[q];
      const float v = (1.0f - b2) * (gt * gt) + b2 * vv[q];
      mv[q] = m;
      vv[q] = v;
      pv[q] = pv[q] + (-lr) * ((m / bc1) / (sqrtf(v / bc2) + eps));
    }
    softmaxq(pv, Q, Tn, sv);
    for (int q = 0; q < Q; ++q) {
      p[r * Q + q] = pv[q];
      mu[r * Q + q] = mv[q];
      nu[r * Q + q] = vv[q];
      s_out[r * Q + q] = sv[q];
    }
  }
}

// Q = 4 (16-B rows): one row per thread over a full grid, every stream
// nontemporal -- 1.63 GB per C5 step touched once, so it should not
// displace anything in L2 / MALL (C5: 329 -> 272 us, 4.9 -> 6.0 TB/s; two or
// four rows per thread, or temporal accesses, were slower: DESIGN §9)
typedef float fv4 __attribute__((ext_vector_type(4)));
#ifndef TREX_ADAM_BLOCK
#define TREX_ADAM_BLOCK 256
#endif
constexpr int kAdamBlock = TREX_ADAM_BLOCK;  // threads per block of the Q = 4 ancestors' pass
__global__ __launch_bounds__(kAdamBlock) void adam_seq_update4_kernel(
    const fv4* __restrict__ ds, int64_t rows, float T, float Tn, fv4* __restrict__ p,
    fv4* __restrict__ mu, fv4* __restrict__ nu, float lr, float b1, float b2, float eps,
    float bc1, float bc2, fv4* __restrict__ s_out, const StepState* __restrict__ ss) {
  if (ss) {
    bc1 = ss->bc1;
    bc2 = ss->bc2;
    T = ss->T;
    Tn = ss->Tn;
  }
  const int64_t r = (int64_t)blockIdx.x * kAdamBlock + threadIdx.x;
  if (r >= rows) return;
  const fv4 d = __builtin_nontemporal_load(ds + r), a = __builtin_nontemporal_load(p + r);
  const fv4 m = __builtin_nontemporal_load(mu + r), v = __builtin_nontemporal_load(nu + r);
  float p4[4], g4[4], m4[4], v4[4], s4[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    p4[q] = a[q];
    g4[q] = d[q];
    m4[q] = m[q];
    v4[q] = v[q];
  }
  adam_seq_row4(g4, p4, m4, v4, T, Tn, lr, b1, b2, eps, bc1, bc2, s4);
  __builtin_nontemporal_store((fv4){p4[0], p4[1], p4[2], p4[3]}, p + r);
  __builtin_nontemporal_store((fv4){m4[0], m4[1], m4[2], m4[3]}, mu + r);
  __builtin_nontemporal_store((fv4){v4[0], v4[1], v4[2], v4[3]}, nu + r);
  __builtin_nontemporal_store((fv4){s4[0], s4[1], s4[2], s4[3]}, s_out + r);
}

int grid_for(int64_t n, int per = 256, int cap = 8192);

// x3p operands: rows x cols of X (row stride ldx) -> split_x3_group layout,
// ldo f32-equivalent columns per row (groups past cols are zero)
__global__ __launch_bounds__(256) void split_x3_kernel(const float* __restrict__ X, int rows,
                                                      int cols, int ldx, float s,
                                                      u32x4* __restrict__ out, int ldo) {
  const int G = ldo / 4;
  const int64_t n = (int64_t)rows * G;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int row = (int)(t / G), c = 4 * (int)(t % G);
    const float* x = X + (size_t)row * ldx;
    out[t] = split_x3_group(c < cols ? x[c] : 0.0f, c + 1 < cols ? x[c + 1] : 0.0f,
                            c + 2 < cols ? x[c + 2] : 0.0f, c + 3 < cols ? x[c + 3] : 0.0f, s);
  }
}

// the Q = 4 ancestors' pass writing the next S rows pre-split (x3p)
__global__ __launch_bounds__(kAdamBlock) void adam_seq_update4_x3p_kernel(
    const fv4* __restrict__ ds, int64_t rows, float T, float Tn, fv4* __restrict__ p,
    fv4* __restrict__ mu, fv4* __restrict__ nu, float lr, float b1, float b2, float eps,
    float bc1, float bc2, float sx, fv4* __restrict__ s_out, const StepState* __restrict__ ss) {
  if (ss) {
    bc1 = ss->bc1;
    bc2 = ss->bc2;
    T = ss->T;
    Tn = ss->Tn;
  }
  const int64_t r = (int64_t)blockIdx.x * kAdamBlock + threadIdx.x;
  if (r >= rows) return;
  const fv4 d = __builtin_nontemporal_load(ds + r), a = __builtin_nontemporal_load(p + r);
  const fv4 m = __builtin_nontemporal_load(mu + r), v = __builtin_nontemporal_load(nu + r);
  float p4[4], g4[4], m4[4], v4[4], s4[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    p4[q] = a[q];
    g4[q] = d[q];
    m4[q] = m[q];
    v4[q] = v[q];
  }
  adam_seq_row4(g4, p4, m4, v4, T, Tn, lr, b1, b2, eps, bc1, bc2, s4);
  __builtin_nontemporal_store((fv4){p4[0], p4[1], p4[2], p4[3]}, p + r);
  __builtin_nontemporal_store((fv4){m4[0], m4[1], m4[2], m4[3]}, mu + r);
  __builtin_nontemporal_store((fv4){v4[0], v4[1], v4[2], v4[3]}, nu + r);
#ifndef TREX_S16_NT
  // the next S rows (pre-split) stay cacheable: the next step's Gram and MF
  // read them (C5 x3 step 0.640-0.652 -> 0.624-0.628 ms same box, PERFLOG)
  s_out[r] = __builtin_bit_cast(fv4, split_x3_group(s4[0], s4[1], s4[2], s4[3], sx));
#else
  __builtin_nontemporal_store(__builtin_bit_cast(fv4, split_x3_group(s4[0], s4[1], s4[2], s4[3], sx)),
                              s_out + r);
#endif
}

void launch_adam_seq(const float* ds, int64_t rows, int Q, float T, float Tn, float* p, float* mu,
                     float* nu, float lr, float b1, float b2, float eps, float bc1, float bc2,
                     float* s_out, const StepState* ss, hipStream_t st) {
  const bool al = ((reinterpret_cast<uintptr_t>(ds) | reinterpret_cast<uintptr_t>(p) |
                    reinterpret_cast<uintptr_t>(mu) | reinterpret_cast<uintptr_t>(nu) |
                    reinterpret_cast<uintptr_t>(s_out)) & 15) == 0;
  if (Q == 4 && al && rows <= 0x7FFFFFFFLL * 256)
    hipLaunchKernelGGL(adam_seq_update4_kernel, dim3((unsigned)((rows + kAdamBlock - 1) / kAdamBlock)), dim3(kAdamBlock), 0,
                       st, reinterpret_cast<const fv4*>(ds), rows, T, Tn,
                       reinterpret_cast<fv4*>(p), reinterpret_cast<fv4*>(mu),
                       reinterpret_cast<fv4*>(nu), lr, b1, b2, eps, bc1, bc2,
                       reinterpret_cast<fv4*>(s_out), ss);
  else
    hipLaunchKernelGGL(adam_seq_update_kernel, dim3(grid_for(rows)), dim3(256), 0, st, ds, rows, Q,
                       T, Tn, p, mu, nu, lr, b1, b2, eps, bc1, bc2, s_out, ss);
}

__global__ __launch_bounds__(256) void identity_kernel(int N, float* __restrict__ A) {
  const size_t total = (size_t)N * N;
  for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (size_t)gridDim.x * 256)
    A[t] = (t / N == t % N) ? 1.0f : 0.0f;
}

// discretize_tree_topology: one_hot(argmax(A[i]), n_nodes), first index on ties
__global__ __launch_bounds__(256) void discretize_kernel(const float* __restrict__ A, int ncols,
                                                        int n_nodes, float* __restrict__ out) {
  __shared__ float bv[256];
  __shared__ int bi[256];
  const int i = blockIdx.x;
  float best = -INFINITY;
  int arg = 0x7FFFFFFF;
  for (int j = threadIdx.x; j < ncols; j += 256) {
    const float v = A[(size_t)i * ncols + j];
    if (v > best || (v == best && j < arg)) { best = v; arg = j; }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = arg;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      const float v = bv[threadIdx.x + w];
      const int k = bi[threadIdx.x + w];
      if (v > bv[threadIdx.x] || (v == bv[threadIdx.x] && k < bi[threadIdx.x])) {
        bv[threadIdx.x] = v;
        bi[threadIdx.x] = k;
      }
    }
    __syncthreads();
  }
  const int a = bi[0] == 0x7FFFFFFF ? 0 : bi[0];
  for (int j = threadIdx.x; j < n_nodes; j += 256) out[(size_t)i * n_nodes + j] = (j == a) ? 1.0f : 0.0f;
}

int grid_for(int64_t n, int per, int cap) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, cap));
}

}  // namespace
}  // namespace trex

using namespace trex;

extern "C" int trex_tree_update_seq(const float* x, int n_anc, int L, int Q, float T, float* s,
                                    void* stream) {
  if (!x || !s || n_anc < 0 || L <= 0 || Q <= 0)
    return set_error(TREX_E_ARG, "trex_tree_update_seq: bad arguments");
  const int64_t rows = (int64_t)n_anc * L;
  if (rows == 0) return TREX_OK;
  hipLaunchKernelGGL(update_seq_kernel, dim3(grid_for(rows)), dim3(256), 0, (hipStream_t)stream,
                     x, rows, Q, T, s);
  return tree_hip_check("trex_tree_update_seq");
}

extern "C" int trex_tree_update_seq_bwd(const float* s, const float* ds, int n_anc, int L, int Q,
                                        float T, float* dx, void* stream) {
  if (!s || !ds || !dx || n_anc < 0 || L <= 0 || Q <= 0)
    return set_error(TREX_E_ARG, "trex_tree_update_seq_bwd: bad arguments");
  const int64_t rows = (int64_t)n_anc * L;
  if (rows == 0) return TREX_OK;
  hipLaunchKernelGGL(update_seq_bwd_kernel, dim3(grid_for(rows)), dim3(256), 0,
                     (hipStream_t)stream, s, ds, rows, Q, T, dx);
  return tree_hip_check("trex_tree_update_seq_bwd");
}

extern "C" int trex_tree_update_tree(const float* theta, const float* noise, const float* gates,
                                     int N, int n_anc, float T, float* A, void* stream) {
  if (!A || N < 2 || n_anc < 0 || n_anc >= N || !pos_finite_f32(T))
    return set_error(TREX_E_ARG, "trex_tree_update_tree: bad arguments");
  if (n_anc > 0 && !theta) return set_error(TREX_E_ARG, "trex_tree_update_tree: theta is NULL");
  if (n_anc == 0) {  // tree.py:68-69: identity
    hipLaunchKernelGGL(identity_kernel, dim3(grid_for((int64_t)N * N)), dim3(256), 0,
                       (hipStream_t)stream, N, A);
    return tree_hip_check("trex_tree_update_tree");
  }
  hipLaunchKernelGGL(update_tree_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, theta, noise,
                     gates, N, n_anc, T, A);
  return tree_hip_check("trex_tree_update_tree");
}

extern "C" int trex_tree_update_tree_bwd(const float* A, const float* dA, const float* gates,
                                         int N, int n_anc, float T, float* dtheta, void* stream) {
  if (!A || !dA || !dtheta || N < 2 || n_anc <= 0 || n_anc >= N || !pos_finite_f32(T))
    return set_error(TREX_E_ARG, "trex_tree_update_tree_bwd: bad arguments");
  hipLaunchKernelGGL(update_tree_bwd_kernel, dim3(N - 1), dim3(256), 0, (hipStream_t)stream, A,
                     dA, gates, N, n_anc, T, dtheta);
  return tree_hip_check("trex_tree_update_tree_bwd");
}

namespace {
struct GramPlan {
  int ntile, npairs, ksplit, kslice;
};
GramPlan gram_plan(int N, int64_t K, bool symmetric = false, int t0 = 0) {
  GramPlan g;
  g.ntile = (N + 63) / 64;
  // workspace is sized for the full (non-symmetric) tile set
  if (symmetric) {
    g.npairs = 0;
    for (int a = 0; a < g.ntile; ++a) g.npairs += sym_row_len(a, g.ntile, t0);
  } else {
    g.npairs = g.ntile * g.ntile;
  }
  // enough waves to fill 256 CUs several times; slices multiple of 32
  int ks = (int)std::max<int64_t>(1, std::min<int64_t>(256, (4096 + g.npairs - 1) / g.npairs));
  ks = (ks + 7) / 8 * 8;
  int64_t slice = (K + ks - 1) / ks;
  slice = (slice + 31) / 32 * 32;
  g.kslice = (int)std::max<int64_t>(32, slice);
  g.ksplit = (int)((K + g.kslice - 1) / g.kslice);
  return g;
}

// v3 plan (symmetric, N <= 512, K % 4 == 0: 16-B aligned rows; a ragged
// last 16-column chunk is zero-masked in the kernel): 32-row strips, tiles per
// group of 8 waves x 13, about one workgroup per CU
struct Gram3Plan {
  int ns, t0s, ntiles, ngroups, ksplit, nchunks;
};
Gram3Plan gram3_plan(int N, int64_t K, int t0s) {
  Gram3Plan g;
  g.ns = (N + 31) / 32;
  g.t0s = t0s;
  g.ntiles = 0;
  for (int a = 0; a < g.ns; ++a) g.ntiles += sym_row_len(a, g.ns, t0s);
  g.ngroups = std::max(1, (g.ntiles + kG3Waves * kG3Tiles - 1) / (kG3Waves * kG3Tiles));
  g.nchunks = (int)((K + 15) / 16);
  g.ksplit = std::max(1, std::min(g.nchunks, std::max(1, 256 / g.ngroups)));
  return g;
}
// v5: ngroups = ceil(ntiles / 64), T = tiles per wave; ksplit a multiple of
// 8 (the XCD pairing of a split's groups), about one workgroup per CU
Gram3Plan gram5_plan(int N, int64_t K, int t0s, int* T, int W = kG5Waves) {
  Gram3Plan g = gram3_plan(N, K, t0s);
  const int maxt = W == 8 ? 8 : kG5MaxTiles;
  g.ngroups = std::max(1, (g.ntiles + W * maxt - 1) / (W * maxt));
  *T = std::max(1, (g.ntiles + W * g.ngroups - 1) / (W * g.ngroups));
  int ks = std::max(1, 256 / g.ngroups);
  ks = std::max(8, ks / 8 * 8);
  g.ksplit = std::max(1, std::min(g.nchunks, ks));
  return g;
}
// kernel version per precision: f32 -> v5 (one wave per SIMD: the 64-cycle
// f32 MFMAs fill the pipe; 587 -> 397 us at C5), x3 -> v3 (two waves per
// SIMD: the f16 MFMA chains need the second wave; v5 measured 231 vs 152
// us).  TREX_GRAM=3 / 5 forces one version for both (A/B).
int gram_version(bool x3) {
  const char* e = std::getenv("TREX_GRAM");
  if (e && (std::atoi(e) == 3 || std::atoi(e) == 5 || std::atoi(e) == 6)) return std::atoi(e);
  return x3 ? 3 : 5;
}
bool gram3_ok(int N, int64_t K) { return N <= kG3Rows && K % 4 == 0 && (int64_t)N * K * 4 < 0x7FFFFFF0LL; }
}  // namespace

namespace {
// split-K partial buffer: the larger of the symmetric and full tile plans
int64_t part_bytes(int N, int64_t K) {
  int64_t b = 0;
  for (bool sym : {true, false}) {
    const GramPlan g = gram_plan(N, K, sym);
    b = std::max<int64_t>(b, (int64_t)((g.ksplit + 7) / 8 * 8) * g.npairs * 4096 * 4);
  }
  if (gram3_ok(N, K)) {
    // every skip (t0s) the v3 path can be given: more skipped tiles can
    // mean fewer groups and so more splits
    const int ns = (N + 31) / 32;
    for (int t0s = 0; t0s <= ns; ++t0s) {
      int T5;
      for (const Gram3Plan& g : {gram3_plan(N, K, t0s), gram5_plan(N, K, t0s, &T5),
                                 gram5_plan(N, K, t0s, &T5, 8)})
        b = std::max<int64_t>(b, (int64_t)g.ksplit * g.ntiles * 4096);
    }
  }
  return b;
}
}  // namespace

extern "C" int64_t trex_tree_workspace_bytes(int N, int64_t K) {
  if (N <= 0 || K <= 0) return 0;
  const int64_t part = part_bytes(N, K);
  const int64_t mats = (int64_t)N * N * 4 * 2;   // G, M
  const int64_t rows = (int64_t)N * 8 * 2 + 8192 * 8;  // row losses / E / norm parts
  return part + mats + rows + 1024;
}

namespace {
// power of two s with max_abs * s <= 2^14 (f16 split headroom)
float split_scale(float max_abs) {
  if (!pos_finite_f32(max_abs)) return 1.0f;
  return std::ldexp(1.0f, 14 - (int)std::ceil(std::log2((double)max_abs)));
}

// x3_max > 0: f16x3 split products with operands bounded by x3_max
// x3_max > 0: f16x3 split products with operands bounded by x3_max
int gram(const float* X, const float* Y, int N, int64_t K, int symmetric, float* G, float* part,
         hipStream_t st, int t0 = 0, float x3_max = 0.0f, bool pre = false, int lzs = 0,
         const uint8_t* codes = nullptr) {
  const GramPlan g = gram_plan(N, K, symmetric != 0, t0);
  if (g.npairs == 0) return TREX_OK;
  const int ks8 = (g.ksplit + 7) / 8 * 8;
  const int blocks = g.npairs * ks8;
  // v5 serves both precisions; v3 (TREX_GRAM=3) only the x3 one
  const bool x3 = x3_max > 0.0f;
  const int gv = pre ? 3 : gram_version(x3);  // pre-split operands: the v3 kernel
  if (pre && !(x3 && symmetric && X == Y && gram3_ok(N, K)))
    return set_error(TREX_E_UNSUPPORTED, "gram: no pre-split kernel for this shape");
  if (symmetric && X == Y && gram3_ok(N, K) && (x3 || gv >= 5)) {
    int T5 = 0;
    const bool v5 = gv >= 5;
    const int W = (gv == 6 && x3) ? 8 : kG5Waves;
    const Gram3Plan p = v5 ? gram5_plan(N, K, 2 * t0, &T5, W) : gram3_plan(N, K, 2 * t0);
    if (p.ntiles == 0) return TREX_OK;
    static const bool lds_set = [] {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gram_kernel3<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kG3Lds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gram_kernel3<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kG3Lds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gram_kernel3<true, 1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kG3Lds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gram_kernel3<true, 2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kG3Lds);
      return true;
    }();
    (void)lds_set;
    const float sc = x3 ? split_scale(x3_max) : 1.0f;
    if (v5) {
      const dim3 grid(((p.ksplit + 7) / 8 * 8) * p.ngroups);
      static const bool set5 = [] {
        for (const void* f : {reinterpret_cast<const void*>(gram_kernel5<4, true>),
                              reinterpret_cast<const void*>(gram_kernel5<8, true>),
                              reinterpret_cast<const void*>(gram_kernel5<10, true>),
                              reinterpret_cast<const void*>(gram_kernel5<12, true>),
                              reinterpret_cast<const void*>(gram_kernel5<13, true>),
                              reinterpret_cast<const void*>(gram_kernel5<16, true>),
                              reinterpret_cast<const void*>(gram_kernel5<4, false>),
                              reinterpret_cast<const void*>(gram_kernel5<8, false>),
                              reinterpret_cast<const void*>(gram_kernel5<10, false>),
                              reinterpret_cast<const void*>(gram_kernel5<12, false>),
                              reinterpret_cast<const void*>(gram_kernel5<13, false>),
                              reinterpret_cast<const void*>(gram_kernel5<16, false>)})
          (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kG3Lds);
        return true;
      }();
      (void)set5;
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(W * kWave), kG3Lds, st, X, N, (int)K, p.ns,
                           p.t0s, p.ntiles, p.ngroups, p.ksplit, p.nchunks, x3 ? sc : 1.0f, part);
      };
      static const bool set6 = [] {
        for (const void* f : {reinterpret_cast<const void*>(gram_kernel5<4, true, 8>),
                              reinterpret_cast<const void*>(gram_kernel5<6, true, 8>),
                              reinterpret_cast<const void*>(gram_kernel5<7, true, 8>),
                              reinterpret_cast<const void*>(gram_kernel5<8, true, 8>)})
          (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kG3Lds);
        return true;
      }();
      (void)set6;
      if (x3 && W == 8) {
        if (T5 <= 4) go(gram_kernel5<4, true, 8>);
        else if (T5 <= 6) go(gram_kernel5<6, true, 8>);
        else if (T5 <= 7) go(gram_kernel5<7, true, 8>);
        else go(gram_kernel5<8, true, 8>);
      } else if (x3) {
        if (T5 <= 4) go(gram_kernel5<4, true>);
        else if (T5 <= 8) go(gram_kernel5<8, true>);
        else if (T5 <= 10) go(gram_kernel5<10, true>);
        else if (T5 <= 12) go(gram_kernel5<12, true>);
        else if (T5 <= 13) go(gram_kernel5<13, true>);
        else go(gram_kernel5<16, true>);
      } else {
        if (T5 <= 4) go(gram_kernel5<4, false>);
        else if (T5 <= 8) go(gram_kernel5<8, false>);
        else if (T5 <= 10) go(gram_kernel5<10, false>);
        else if (T5 <= 12) go(gram_kernel5<12, false>);
        else if (T5 <= 13) go(gram_kernel5<13, false>);
        else go(gram_kernel5<16, false>);
      }
    } else {
      auto go3 = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(p.ksplit * p.ngroups), dim3(kG3Waves * kWave), kG3Lds, st, X,
                           N, (int)K, p.ns, p.t0s, p.ntiles, p.ngroups, p.ksplit, p.nchunks, sc,
                           part, lzs, codes);
      };
      // code rows by compile-time passes of 128 rows (C5: 256 leaves, 2)
      const int ncp = (pre && codes && lzs > 0 && (32 * lzs) % kG3Rows4 == 0) ? 32 * lzs / kG3Rows4 : 0;
      if (pre && ncp == 1) go3(gram_kernel3<true, 1>);
      else if (pre && ncp == 2) go3(gram_kernel3<true, 2>);
      else if (pre) go3(gram_kernel3<true>);
      else go3(gram_kernel3<false>);
    }
    hipLaunchKernelGGL(gram3_reduce_kernel, dim3(p.ntiles * 16), dim3(256), 0, st, part, N, p.ns,
                       p.t0s, p.ntiles, p.ksplit, G);
    return tree_hip_check("gram");
  }
  if (K % 16 == 0 && x3_max > 0.0f) {
    const float sc = split_scale(x3_max);
    hipLaunchKernelGGL(gram_kernel2<true>, dim3(blocks), dim3(kWave), 0, st, X, Y, N, (int)K,
                       g.ntile, g.npairs, symmetric, t0, g.ksplit, g.kslice, part, sc, sc);
  } else if (K % 16 == 0)
    hipLaunchKernelGGL(gram_kernel2<false>, dim3(blocks), dim3(kWave), 0, st, X, Y, N, (int)K, g.ntile,
                       g.npairs, symmetric, t0, g.ksplit, g.kslice, part);
  else
    hipLaunchKernelGGL(gram_kernel, dim3(blocks), dim3(kWave), 0, st, X, Y, N, (int)K, g.ntile,
                       g.npairs, symmetric, t0, g.ksplit, g.kslice, part);
  const size_t total = (size_t)g.npairs * 4096;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3(grid_for((int64_t)total)), dim3(256), 0, st, part, N,
                     g.ntile, g.npairs, g.ksplit, symmetric, t0, G);
  return tree_hip_check("gram");
}
}  // namespace

extern "C" int trex_tree_surrogate(const float* S, const float* A, int N, int64_t K, float* loss,
                                   float* dS, float* dA, float* G_out, void* workspace,
                                   int64_t workspace_bytes, void* stream) {
  if (!S || !A || !loss || !workspace || N <= 0 || K <= 0 || K > 0x7FFFFFFF)
    return set_error(TREX_E_ARG, "trex_tree_surrogate: bad arguments");
  if (workspace_bytes < trex_tree_workspace_bytes(N, K))
    return set_error(TREX_E_ARG, "trex_tree_surrogate: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  char* w = static_cast<char*>(workspace);
  float* part = reinterpret_cast<float*>(w);
  w += part_bytes(N, K);
  float* G = reinterpret_cast<float*>(w);
  w += (int64_t)N * N * 4;
  float* M = reinterpret_cast<float*>(w);
  w += (int64_t)N * N * 4;
  double* rowloss = reinterpret_cast<double*>(w);
  if (N <= kSurSmallN && (int64_t)N * K <= kSurSmallNK) {
    hipLaunchKernelGGL(surrogate_small_kernel, dim3(1), dim3(1024), 0, st, S, A, N, (int)K, loss,
                       dS, dA, G_out);
    return tree_hip_check("trex_tree_surrogate");
  }
  if (int e = gram(S, S, N, K, 1, G, part, st)) return e;
  hipLaunchKernelGGL(surrogate_combine_kernel, dim3(N), dim3(256), 0, st, A, G, N, dA,
                     dS ? M : nullptr, rowloss);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, st, rowloss, N, 1.0f, loss, 0,
                     (const StepState*)nullptr);
  if (dS) {
    const int nrowt = (N + 63) / 64;
    const int ncolb = (int)((K + 63) / 64);
    const int blocks = nrowt * ((ncolb + 7) / 8 * 8);
    hipLaunchKernelGGL(mf_kernel2<false>, dim3(blocks), dim3(kWave), 0, st, M, S, N, (int)K, 0, N, nrowt, ncolb,
                       dS);
  }
  if (G_out &&
      hipMemcpyAsync(G_out, G, sizeof(float) * (size_t)N * N, hipMemcpyDeviceToDevice, st) !=
          hipSuccess)
    return tree_hip_check("trex_tree_surrogate(G)");
  return tree_hip_check("trex_tree_surrogate");
}

extern "C" int trex_tree_soft_cost(const float* S, const float* A, const float* C, int ckind,
                                   int N, int L, int Q, float* loss, float* W_scratch,
                                   void* workspace, int64_t workspace_bytes, void* stream) {
  const int64_t K = (int64_t)L * Q;
  if (!S || !A || !loss || !workspace || N <= 0 || L <= 0 || Q <= 0 || ckind < 0 || ckind > 2 ||
      (ckind > 0 && !C) || (ckind > 0 && !W_scratch))
    return set_error(TREX_E_ARG, "trex_tree_soft_cost: bad arguments");
  if (workspace_bytes < trex_tree_workspace_bytes(N, K))
    return set_error(TREX_E_ARG, "trex_tree_soft_cost: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  char* w = static_cast<char*>(workspace);
  float* part = reinterpret_cast<float*>(w);
  w += part_bytes(N, K);
  float* G = reinterpret_cast<float*>(w);
  w += (int64_t)N * N * 8;
  double* rowloss = reinterpret_cast<double*>(w);
  const float* Wp = S;
  if (ckind > 0) {
    const int64_t rows = (int64_t)N * L;
    hipLaunchKernelGGL(weight_seq_kernel, dim3(grid_for(rows)), dim3(256), 0, st, S, rows, Q, C,
                       ckind, W_scratch);
    Wp = W_scratch;
  }
  // G[i][j] = <S_i, W_j> (not symmetric for a general C): all tile pairs
  if (int e = gram(S, Wp, N, K, ckind == 0 ? 1 : 0, G, part, st)) return e;
  hipLaunchKernelGGL(soft_combine_kernel, dim3(N), dim3(256), 0, st, A, G, N, rowloss);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, st, rowloss, N, 1.0f, loss, 0,
                     (const StepState*)nullptr);
  return tree_hip_check("trex_tree_soft_cost");
}

extern "C" int trex_tree_constraint(const float* A, int N, float scale, float grad_scale,
                                    float* loss, int accumulate, float* dA, void* workspace,
                                    void* stream) {
  if (!A || !loss || !workspace || N < 3)
    return set_error(TREX_E_ARG, "trex_tree_constraint: bad arguments");
  const int n_anc = (N - 1) / 2;
  hipStream_t st = (hipStream_t)stream;
  double* colloss = static_cast<double*>(workspace);
  hipLaunchKernelGGL(constraint_kernel, dim3(n_anc), dim3(256), 0, st, A, N, scale, grad_scale,
                     colloss, dA, (const StepState*)nullptr);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, st, colloss, n_anc, grad_scale,
                     loss, accumulate, (const StepState*)nullptr);
  return tree_hip_check("trex_tree_constraint");
}

extern "C" int trex_tree_constraint_dev(const float* A, int N, float scale, const void* state,
                                        float* loss, int accumulate, float* dA, void* workspace,
                                        void* stream) {
  if (!A || !loss || !workspace || !state || N < 3)
    return set_error(TREX_E_ARG, "trex_tree_constraint_dev: bad arguments");
  const int n_anc = (N - 1) / 2;
  hipStream_t st = (hipStream_t)stream;
  double* colloss = static_cast<double*>(workspace);
  const StepState* ss = static_cast<const StepState*>(state);
  hipLaunchKernelGGL(constraint_kernel, dim3(n_anc), dim3(256), 0, st, A, N, scale, 0.0f, colloss,
                     dA, ss);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, st, colloss, n_anc, 0.0f, loss,
                     accumulate, ss);
  return tree_hip_check("trex_tree_constraint_dev");
}

extern "C" int trex_tree_compute_cost(const float* S, const float* A, const float* subst, int N,
                                      int L, int Q, float* cost, void* workspace, void* stream) {
  if (!S || !A || !subst || !cost || !workspace || N < 2 || L <= 0 || Q <= 0)
    return set_error(TREX_E_ARG, "trex_tree_compute_cost: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  double* rowcost = static_cast<double*>(workspace);
  // rows 0..N-2 only ([:-1] in tree.py:296)
  hipLaunchKernelGGL(compute_cost_kernel, dim3(N - 1), dim3(256), 0, st, S, A, subst, N, L, Q,
                     rowcost);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, st, rowcost, N - 1, 1.0f, cost, 0,
                     (const StepState*)nullptr);
  return tree_hip_check("trex_tree_compute_cost");
}

extern "C" int trex_adam_step(float* params, const float* grads, float* mu, float* nu, int64_t n,
                              int count, float lr, float b1, float b2, float eps,
                              const double* grad_sq_norm_parts, int n_parts, float clip_norm,
                              void* stream) {
  if (!params || !grads || !mu || !nu || n < 0 || count < 1)
    return set_error(TREX_E_ARG, "trex_adam_step: bad arguments");
  const float bc1 = bias_corr(b1, count);
  const float bc2 = bias_corr(b2, count);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, params,
                     grads, mu, nu, n, lr, b1, b2, eps, bc1, bc2, grad_sq_norm_parts, n_parts,
                     clip_norm, (const StepState*)nullptr);
  return tree_hip_check("trex_adam_step");
}

extern "C" int trex_step_state_bytes(void) { return (int)sizeof(StepState); }

extern "C" int trex_step_advance(void* state, float b1, float b2, const float* temps,
                                 int64_t n_temps, void* stream) {
  if (!state || (temps && n_temps <= 0))
    return set_error(TREX_E_ARG, "trex_step_advance: bad arguments");
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream,
                     static_cast<StepState*>(state), b1, b2, temps, n_temps);
  return tree_hip_check("trex_step_advance");
}

extern "C" int trex_tree_update_tree_bwd_adam(const float* A, const float* dA, const float* gates,
                                              int N, int n_anc, float T, float* dtheta,
                                              float* params, float* mu, float* nu, int count,
                                              const void* state, float lr, float b1, float b2,
                                              float eps, void* stream) {
  if (!A || !dA || !params || !mu || !nu || N < 2 || n_anc <= 0 || n_anc >= N ||
      !pos_finite_f32(T) || (!state && count < 1))
    return set_error(TREX_E_ARG, "trex_tree_update_tree_bwd_adam: bad arguments");
  const float bc1 = state ? 1.0f : bias_corr(b1, count);
  const float bc2 = state ? 1.0f : bias_corr(b2, count);
  hipLaunchKernelGGL(update_tree_bwd_adam_kernel, dim3(N - 1), dim3(256), 0, (hipStream_t)stream,
                     A, dA, gates, N, n_anc, T, dtheta, params, mu, nu, lr, b1, b2, eps, bc1, bc2,
                     static_cast<const StepState*>(state));
  return tree_hip_check("trex_tree_update_tree_bwd_adam");
}

extern "C" int trex_adam_step_dev(float* params, const float* grads, float* mu, float* nu,
                                  int64_t n, const void* state, float lr, float b1, float b2,
                                  float eps, const double* grad_sq_norm_parts, int n_parts,
                                  float clip_norm, void* stream) {
  if (!params || !grads || !mu || !nu || n < 0 || !state)
    return set_error(TREX_E_ARG, "trex_adam_step_dev: bad arguments");
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, params,
                     grads, mu, nu, n, lr, b1, b2, eps, 1.0f, 1.0f, grad_sq_norm_parts, n_parts,
                     clip_norm, static_cast<const StepState*>(state));
  return tree_hip_check("trex_adam_step_dev");
}

extern "C" int trex_optax_step(int kind, float* params, const float* grads, float* state1,
                               float* state2, int64_t n, int count, float lr, float b1, float b2,
                               float eps, float weight_decay, const double* grad_sq_norm_parts,
                               int n_parts, float clip_norm, void* stream) {
  if (kind < 0 || kind > 3 || !params || !grads || n < 0 || count < 1 ||
      ((kind != 3) && !state1) || ((kind != 2) && !state2))
    return set_error(TREX_E_ARG, "trex_optax_step: bad arguments");
  const float bc1 = bias_corr(b1, count);
  const float bc2 = bias_corr(b2, count);
  hipLaunchKernelGGL(optax_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, kind,
                     params, grads, state1, state2, n, lr, b1, b2, eps, weight_decay, bc1, bc2,
                     grad_sq_norm_parts, n_parts, clip_norm, (const StepState*)nullptr);
  return tree_hip_check("trex_optax_step");
}

extern "C" int trex_optax_step_dev(int kind, float* params, const float* grads, float* state1,
                                   float* state2, int64_t n, const void* state, float lr, float b1,
                                   float b2, float eps, float weight_decay,
                                   const double* grad_sq_norm_parts, int n_parts, float clip_norm,
                                   void* stream) {
  if (kind < 0 || kind > 3 || !params || !grads || n < 0 || !state ||
      ((kind != 3) && !state1) || ((kind != 2) && !state2))
    return set_error(TREX_E_ARG, "trex_optax_step_dev: bad arguments");
  hipLaunchKernelGGL(optax_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, kind,
                     params, grads, state1, state2, n, lr, b1, b2, eps, weight_decay, 1.0f, 1.0f,
                     grad_sq_norm_parts, n_parts, clip_norm, static_cast<const StepState*>(state));
  return tree_hip_check("trex_optax_step_dev");
}

extern "C" int trex_adam_seq_step(const float* s_anc, const float* ds_anc, int n_anc, int L,
                                  int Q, float temperature, float* params, float* mu, float* nu,
                                  int count, float lr, float b1, float b2, float eps,
                                  float* grads_out, void* stream) {
  if (!s_anc || !ds_anc || !params || !mu || !nu || n_anc <= 0 || L <= 0 || Q < 2 || Q > 32 ||
      count < 1 || !pos_finite_f32(temperature))
    return set_error(TREX_E_ARG, "trex_adam_seq_step: bad arguments");
  const float bc1 = bias_corr(b1, count);
  const float bc2 = bias_corr(b2, count);
  const int64_t rows = (int64_t)n_anc * L;
  const bool al = ((reinterpret_cast<uintptr_t>(s_anc) | reinterpret_cast<uintptr_t>(ds_anc) |
                    reinterpret_cast<uintptr_t>(params) | reinterpret_cast<uintptr_t>(mu) |
                    reinterpret_cast<uintptr_t>(nu) | reinterpret_cast<uintptr_t>(grads_out)) &
                   15) == 0;
  hipStream_t st = (hipStream_t)stream;
  if (Q == 4 && al)
    hipLaunchKernelGGL(adam_seq_kernel<4>, dim3(grid_for(rows)), dim3(256), 0, st, s_anc, ds_anc,
                       rows, Q, temperature, params, mu, nu, lr, b1, b2, eps, bc1, bc2, grads_out);
  else
    hipLaunchKernelGGL(adam_seq_kernel<0>, dim3(grid_for(rows)), dim3(256), 0, st, s_anc, ds_anc,
                       rows, Q, temperature, params, mu, nu, lr, b1, b2, eps, bc1, bc2, grads_out);
  return tree_hip_check("trex_adam_seq_step");
}

extern "C" int trex_adam_seq_update_step(const float* ds_anc, int n_anc, int L, int Q,
                                         float temperature, float next_temperature,
                                         float* params, float* mu, float* nu, int count, float lr,
                                         float b1, float b2, float eps, float* s_next,
                                         void* stream) {
  if (!ds_anc || !params || !mu || !nu || !s_next || n_anc <= 0 || L <= 0 || Q < 2 || Q > 32 ||
      count < 1 || !pos_finite_f32(temperature) || !pos_finite_f32(next_temperature))
    return set_error(TREX_E_ARG, "trex_adam_seq_update_step: bad arguments");
  const float bc1 = bias_corr(b1, count);
  const float bc2 = bias_corr(b2, count);
  const int64_t rows = (int64_t)n_anc * L;
  launch_adam_seq(ds_anc, rows, Q, temperature, next_temperature, params, mu, nu, lr, b1, b2, eps,
                  bc1, bc2, s_next, nullptr, (hipStream_t)stream);
  return tree_hip_check("trex_adam_seq_update_step");
}

extern "C" int trex_adam_seq_update_step_dev(const float* ds_anc, int n_anc, int L, int Q,
                                             const void* state, float* params, float* mu,
                                             float* nu, float lr, float b1, float b2, float eps,
                                             float* s_next, void* stream) {
  if (!ds_anc || !params || !mu || !nu || !s_next || !state || n_anc <= 0 || L <= 0 || Q < 2 ||
      Q > 32)
    return set_error(TREX_E_ARG, "trex_adam_seq_update_step_dev: bad arguments");
  const int64_t rows = (int64_t)n_anc * L;
  launch_adam_seq(ds_anc, rows, Q, 1.0f, 1.0f, params, mu, nu, lr, b1, b2, eps, 1.0f, 1.0f, s_next,
                  static_cast<const StepState*>(state), (hipStream_t)stream);
  return tree_hip_check("trex_adam_seq_update_step_dev");
}

extern "C" int trex_adam_seq_update_step_x3p(const float* ds_anc, int n_anc, int L, int Q,
                                             float temperature, float next_temperature,
                                             float* params, float* mu, float* nu, int count,
                                             float lr, float b1, float b2, float eps,
                                             const void* state, float max_abs_s, void* s16_next,
                                             void* stream) {
  if (!ds_anc || !params || !mu || !nu || !s16_next || n_anc <= 0 || L <= 0 || Q != 4 ||
      !pos_finite_f32(max_abs_s) ||
      (!state && (count < 1 || !pos_finite_f32(temperature) ||
                  !pos_finite_f32(next_temperature))) ||
      ((reinterpret_cast<uintptr_t>(ds_anc) | reinterpret_cast<uintptr_t>(params) |
        reinterpret_cast<uintptr_t>(mu) | reinterpret_cast<uintptr_t>(nu) |
        reinterpret_cast<uintptr_t>(s16_next)) & 15) != 0)
    return set_error(TREX_E_ARG, "trex_adam_seq_update_step_x3p: bad arguments");
  const int64_t rows = (int64_t)n_anc * L;
  const float bc1 = state ? 1.0f : bias_corr(b1, count);
  const float bc2 = state ? 1.0f : bias_corr(b2, count);
  hipLaunchKernelGGL(adam_seq_update4_x3p_kernel, dim3((unsigned)((rows + kAdamBlock - 1) / kAdamBlock)), dim3(kAdamBlock),
                     0, (hipStream_t)stream, reinterpret_cast<const fv4*>(ds_anc), rows,
                     temperature, next_temperature, reinterpret_cast<fv4*>(params),
                     reinterpret_cast<fv4*>(mu), reinterpret_cast<fv4*>(nu), lr, b1, b2, eps, bc1,
                     bc2, split_scale(max_abs_s), static_cast<fv4*>(s16_next),
                     static_cast<const StepState*>(state));
  return tree_hip_check("trex_adam_seq_update_step_x3p");
}

extern "C" int trex_sq_norm_parts(const float* x, int64_t n, double* parts, int n_parts,
                                  void* stream) {
  if (!x || !parts || n_parts <= 0 || n_parts > 8192)
    return set_error(TREX_E_ARG, "trex_sq_norm_parts: bad arguments");
  hipLaunchKernelGGL(sq_norm_kernel, dim3(n_parts), dim3(256), 0, (hipStream_t)stream, x, n,
                     parts);
  return tree_hip_check("trex_sq_norm_parts");
}

extern "C" int trex_tree_discretize(const float* A, int nrows, int ncols, int n_nodes, float* out,
                                    void* stream) {
  if (!A || !out || nrows <= 0 || ncols <= 0 || n_nodes <= 0)
    return set_error(TREX_E_ARG, "trex_tree_discretize: bad arguments");
  hipLaunchKernelGGL(discretize_kernel, dim3(nrows), dim3(256), 0, (hipStream_t)stream, A, ncols,
                     n_nodes, out);
  return tree_hip_check("trex_tree_discretize");
}

// ---- split surrogate phases (for site-sharded multi-GPU: all-reduce G between
// trex_tree_gram and trex_tree_surrogate_combine) ----
extern "C" int trex_tree_gram_skip(const float* S, int N, int64_t K, int skip_rows, float* G,
                                   void* workspace, int64_t workspace_bytes, void* stream) {
  if (!S || !G || !workspace || N <= 0 || K <= 0 || K > 0x7FFFFFFF || skip_rows < 0 ||
      skip_rows > N)
    return set_error(TREX_E_ARG, "trex_tree_gram_skip: bad arguments");
  if (workspace_bytes < trex_tree_workspace_bytes(N, K))
    return set_error(TREX_E_ARG, "trex_tree_gram_skip: workspace too small");
  return gram(S, S, N, K, 1, G, static_cast<float*>(workspace), (hipStream_t)stream,
              skip_rows / 64);
}

extern "C" int trex_tree_gram_skip_x3(const float* S, int N, int64_t K, int skip_rows,
                                      float max_abs, float* G, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
  if (!S || !G || !workspace || N <= 0 || K <= 0 || K > 0x7FFFFFFF || skip_rows < 0 ||
      skip_rows > N || !pos_finite_f32(max_abs))
    return set_error(TREX_E_ARG, "trex_tree_gram_skip_x3: bad arguments");
  if (K % 4 != 0)
    return set_error(TREX_E_UNSUPPORTED, "trex_tree_gram_skip_x3: K = L*Q must be a multiple of 4");
  if (workspace_bytes < trex_tree_workspace_bytes(N, K))
    return set_error(TREX_E_ARG, "trex_tree_gram_skip_x3: workspace too small");
  return gram(S, S, N, K, 1, G, static_cast<float*>(workspace), (hipStream_t)stream,
              skip_rows / 64, max_abs);
}

extern "C" int trex_tree_gram_mirror(float* G, int N, int row0, void* stream) {
  if (!G || N <= 0 || row0 < 0 || row0 > N)
    return set_error(TREX_E_ARG, "trex_tree_gram_mirror: bad arguments");
  if (row0 == 0 || row0 == N) return TREX_OK;
  const int64_t n = (int64_t)row0 * (N - row0);
  hipLaunchKernelGGL(gram_mirror_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1024)),
                     dim3(256), 0, (hipStream_t)stream, G, N, row0);
  return tree_hip_check("trex_tree_gram_mirror");
}

extern "C" int trex_tree_gram(const float* S, int N, int64_t K, float* G, void* workspace,
                              int64_t workspace_bytes, void* stream) {
  return trex_tree_gram_skip(S, N, K, 0, G, workspace, workspace_bytes, stream);
}

extern "C" int trex_tree_surrogate_constraint(const float* A, const float* G, int N, float scale,
                                              float grad_scale, const void* state, float* loss,
                                              float* dA, float* M, float max_abs_m, void* M16,
                                              int ldm16, void* workspace, void* stream) {
  if (!A || !G || !loss || !dA || !M || !workspace || N < 3 ||
      (M16 && (ldm16 < N || ldm16 % 4 != 0 || !pos_finite_f32(max_abs_m))))
    return set_error(TREX_E_ARG, "trex_tree_surrogate_constraint: bad arguments");
  const int n_anc = (N - 1) / 2;
  hipStream_t st = (hipStream_t)stream;
  double* rowloss = static_cast<double*>(workspace);
  double* colloss = rowloss + N;
  const StepState* ss = static_cast<const StepState*>(state);
  hipLaunchKernelGGL(surrogate_combine_kernel, dim3(N), dim3(256), 0, st, A, G, N, dA, M,
                     rowloss, static_cast<_Float16*>(M16), ldm16,
                     M16 ? split_scale(max_abs_m) : 1.0f);
  hipLaunchKernelGGL(constraint_kernel, dim3(n_anc), dim3(256), 0, st, A, N, scale, grad_scale,
                     colloss, dA, ss);
  hipLaunchKernelGGL(sum_rows2_kernel, dim3(1), dim3(256), 0, st, rowloss, N, colloss, n_anc,
                     grad_scale, loss, ss);
  return tree_hip_check("trex_tree_surrogate_constraint");
}

extern "C" int trex_tree_surrogate_combine(const float* A, const float* G, int N, float* loss,
                                           float* dA, float* M, void* workspace, void* stream) {
  if (!A || !G || !loss || !workspace || N <= 0)
    return set_error(TREX_E_ARG, "trex_tree_surrogate_combine: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  double* rowloss = static_cast<double*>(workspace);
  hipLaunchKernelGGL(surrogate_combine_kernel, dim3(N), dim3(256), 0, st, A, G, N, dA, M,
                     rowloss);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, st, rowloss, N, 1.0f, loss, 0,
                     (const StepState*)nullptr);
  return tree_hip_check("trex_tree_surrogate_combine");
}

namespace {
int mf_x3(const char* fn, const float* M, const float* S, int N, int64_t K, int row0, int nrows,
          float max_abs_m, float max_abs_s, float* dS_rows, const uint8_t* codesR, int lcs,
          void* stream, bool x3, bool pre = false, int ldm = 0);
}  // namespace
extern "C" int trex_tree_mf_rows(const float* M, const float* S, int N, int64_t K, int row0,
                                 int nrows, float* dS_rows, void* stream) {
  if (!M || !S || !dS_rows || N <= 0 || K <= 0 || K > 0x7FFFFFFF || row0 < 0 || nrows <= 0 ||
      row0 + nrows > N)
    return set_error(TREX_E_ARG, "trex_tree_mf_rows: bad arguments");
  if ((int64_t)N * K * 4 > 0x7FFFFFF0LL)
    return set_error(TREX_E_UNSUPPORTED, "trex_tree_mf_rows: S exceeds 2 GiB");
  // v5 f32 (one wave per SIMD, K % 4 == 0: 16-B rows; 525 -> 467 us at C5);
  // TREX_MF=3 or a ragged K: the one-wave-per-tile kernel
  const char* ev = std::getenv("TREX_MF");
  if (K % 4 == 0 && 32LL * K * 4 < 0x7FFFFFF0LL && !(ev && std::atoi(ev) == 3))
    return mf_x3("trex_tree_mf_rows", M, S, N, K, row0, nrows, 1.0f, 1.0f, dS_rows, nullptr, 0,
                 stream, false);
  const int nrowt = (nrows + 63) / 64;
  const int ncolb = (int)((K + 63) / 64);
  const int blocks = nrowt * ((ncolb + 7) / 8 * 8);
  hipLaunchKernelGGL(mf_kernel2<false>, dim3(blocks), dim3(kWave), 0, (hipStream_t)stream, M, S, N,
                     (int)K, row0, nrows, nrowt, ncolb, dS_rows);
  return tree_hip_check("trex_tree_mf_rows");
}

namespace {
// v3 MF launch; codesR / lcs: leaf-code stages (CODES instantiation) or null / 0
int mf_x3(const char* fn, const float* M, const float* S, int N, int64_t K, int row0, int nrows,
          float max_abs_m, float max_abs_s, float* dS_rows, const uint8_t* codesR, int lcs,
          void* stream, bool x3, bool pre, int ldm) {
  if (!pre) ldm = N;
  if (!M || !S || !dS_rows || N <= 0 || K <= 0 || K > 0x7FFFFFFF || row0 < 0 || nrows <= 0 ||
      row0 + nrows > N || !pos_finite_f32(max_abs_m) || !pos_finite_f32(max_abs_s))
    return set_error(TREX_E_ARG, "%s: bad arguments", fn);
  if ((int64_t)N * K * 4 > 0x7FFFFFF0LL)
    return set_error(TREX_E_UNSUPPORTED, "%s: S exceeds 2 GiB", fn);
  // float4 operand loads: rows must start 16-B aligned (the last column tile
  // may be ragged: its columns past K are computed from the next row's data
  // and never stored)
  if (K % 4 != 0)
    return set_error(TREX_E_UNSUPPORTED, "%s: K = L*Q must be a multiple of 4", fn);
  // column tiles per workgroup: fewest rounds x tiles over one workgroup per CU
  const int64_t ct = (K + 31) / 32;
  const int rg = (nrows + 255) / 256;
  int best = 5;
  int64_t best_cost = INT64_MAX;
  for (int tpc : {5, 4}) {
    const int64_t wgs = (ct + tpc - 1) / tpc * rg;
    const int64_t cost = (wgs + cu_count() - 1) / cu_count() * tpc;
    if (cost < best_cost) { best_cost = cost; best = tpc; }
  }
  auto go = [&](auto kernel, int tpc, int lds) {
    if (lds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    const int nch = (int)((ct + tpc - 1) / tpc);
    // one persistent workgroup per CU (per row group)
    const int gx = std::max(1, std::min(nch, std::max(1, cu_count() / rg)));
    hipLaunchKernelGGL(kernel, dim3(gx, rg), dim3(512), lds, (hipStream_t)stream, M, S, N,
                       (int)K, row0, nrows, nch, dS_rows, split_scale(max_abs_m),
                       split_scale(max_abs_s), codesR, lcs, ldm);
  };
  const int lds = 2 * (2 * 32 * 320 + 256 * kMfStride);
  const bool codes = codesR && lcs > 0;
  const char* ev = std::getenv("TREX_MF");
  // v5's dropped stores carry an out-of-bounds voffset plus a row soffset
  // (< 32 K * 4 bytes): kept below 2^31 so the sum cannot wrap in bounds
  const bool v5_ok = 32LL * K * 4 < 0x7FFFFFF0LL;
  if (!x3 && !v5_ok) return set_error(TREX_E_UNSUPPORTED, "%s: K too large for the f32 v5 MF", fn);
  // f32: v5; x3: v3 (v5 measured 242 vs 224 us with leaf codes at C5) unless TREX_MF=5
  if (pre) {  // pre-split operands: the v3 kernel
    if (!x3 || ldm < N || ldm % 32 != 0 || (int64_t)N * ldm * 4 > 0x7FFFFFF0LL)
      return set_error(TREX_E_ARG, "%s: bad pre-split M stride", fn);
    if (best == 5) {
      if (codes) go(mf_kernel3<5, true, true>, 5, lds);
      else go(mf_kernel3<5, false, true>, 5, lds);
    } else {
      if (codes) go(mf_kernel3<4, true, true>, 4, lds);
      else go(mf_kernel3<4, false, true>, 4, lds);
    }
    return tree_hip_check(fn);
  }
  if (v5_ok && (!x3 || (ev && std::atoi(ev) == 5))) {
    // f32: the transposed F slice is CW x 144 B
    const int lds5 = x3 ? lds : 2 * (160 * kMfStride + 256 * kMfStride);
    auto go5 = [&](auto kernel, int tpc) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds5);
      const int nch = (int)((ct + tpc - 1) / tpc);
      const int gx = std::max(1, std::min(nch, std::max(1, cu_count() / rg)));
      hipLaunchKernelGGL(kernel, dim3(gx, rg), dim3(256), lds5, (hipStream_t)stream, M, S, N,
                         (int)K, row0, nrows, nch, dS_rows, x3 ? split_scale(max_abs_m) : 1.0f,
                         x3 ? split_scale(max_abs_s) : 1.0f, codesR, lcs);
    };
    if (!x3) {
      if (best == 5) go5(mf_kernel5<5, false, false>, 5);
      else go5(mf_kernel5<4, false, false>, 4);
    } else if (best == 5) {
      if (codes) go5(mf_kernel5<5, true, true>, 5);
      else go5(mf_kernel5<5, false, true>, 5);
    } else {
      if (codes) go5(mf_kernel5<4, true, true>, 4);
      else go5(mf_kernel5<4, false, true>, 4);
    }
    return tree_hip_check(fn);
  }
  if (best == 5) {
    if (codes) go(mf_kernel3<5, true>, 5, lds);
    else go(mf_kernel3<5, false>, 5, lds);
  } else {
    if (codes) go(mf_kernel3<4, true>, 4, lds);
    else go(mf_kernel3<4, false>, 4, lds);
  }
  return tree_hip_check(fn);
}

// leaf codes of rows [0, lcr): codesR [lcr][L] bytes, the state of each
// exactly one-hot (row, site); 0xFF and *status = 1 otherwise
__global__ __launch_bounds__(256) void leaf_codes_kernel(const float* __restrict__ S, int L, int lcr,
                                                         uint8_t* __restrict__ codesR,
                                                         int* __restrict__ status) {
  const int64_t n = (int64_t)lcr * L;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4*>(S)[t];  // row t / L, site t % L, Q = 4
    const float e[4] = {v.x, v.y, v.z, v.w};
    int ones = 0, idx = 0;
    bool clean = true;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (e[q] == 1.0f) {
        ++ones;
        idx = q;
      } else if (e[q] != 0.0f) {
        clean = false;
      }
    }
    const bool ok = clean && ones == 1;
    codesR[t] = ok ? (uint8_t)idx : (uint8_t)0xFF;
    if (!ok) atomicOr(status, 1);
  }
}
}  // namespace

extern "C" int trex_tree_mf_rows_x3(const float* M, const float* S, int N, int64_t K, int row0,
                                    int nrows, float max_abs_m, float max_abs_s, float* dS_rows,
                                    void* stream) {
  return mf_x3("trex_tree_mf_rows_x3", M, S, N, K, row0, nrows, max_abs_m, max_abs_s, dS_rows,
               nullptr, 0, stream, true);
}

extern "C" int trex_tree_leaf_code_rows(int n_leaf) { return n_leaf >= 32 ? 32 * (n_leaf / 32) : 0; }

extern "C" int64_t trex_tree_leaf_codes_bytes(int n_leaf, int L) {
  const int64_t lcr = trex_tree_leaf_code_rows(n_leaf);
  return (L <= 0 || lcr <= 0) ? 0 : lcr * L;
}

extern "C" int trex_tree_leaf_codes(const float* S, int n_leaf, int L, int Q, void* codes,
                                    int64_t codes_bytes, int* status, void* stream) {
  const int lcr = trex_tree_leaf_code_rows(n_leaf);
  if (!S || !codes || !status || L <= 0 || Q != 4 || lcr <= 0 ||
      (reinterpret_cast<uintptr_t>(S) & 15) != 0)
    return set_error(TREX_E_ARG, "trex_tree_leaf_codes: bad arguments (Q = 4, n_leaf >= 32, 16-B aligned S)");
  if (codes_bytes < trex_tree_leaf_codes_bytes(n_leaf, L))
    return set_error(TREX_E_ARG, "trex_tree_leaf_codes: codes buffer too small");
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(status, 0, sizeof(int), st) != hipSuccess)
    return set_error(TREX_E_HIP, "trex_tree_leaf_codes: memset failed");
  const int64_t n = (int64_t)lcr * L;
  hipLaunchKernelGGL(leaf_codes_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)),
                     dim3(256), 0, st, S, L, lcr, static_cast<uint8_t*>(codes), status);
  return tree_hip_check("trex_tree_leaf_codes");
}

extern "C" int trex_tree_mf_rows_x3_codes(const float* M, const float* S, int N, int64_t K,
                                          int row0, int nrows, float max_abs_m, float max_abs_s,
                                          const void* codes, int64_t codes_bytes, int n_leaf,
                                          int Q, float* dS_rows, void* stream) {
  const int lcr = trex_tree_leaf_code_rows(n_leaf);
  if (!codes || lcr <= 0 || lcr > N || Q != 4 || K % 4 != 0)
    return set_error(TREX_E_ARG, "trex_tree_mf_rows_x3_codes: bad arguments (Q = 4 codes only)");
  // one code byte per (code row, site): the buffer trex_tree_leaf_codes filled
  if (codes_bytes < (int64_t)lcr * (K / Q))
    return set_error(TREX_E_ARG, "trex_tree_mf_rows_x3_codes: codes buffer smaller than "
                                 "trex_tree_leaf_codes_bytes(n_leaf, K / Q)");
  return mf_x3("trex_tree_mf_rows_x3_codes", M, S, N, K, row0, nrows, max_abs_m, max_abs_s,
               dS_rows, static_cast<const uint8_t*>(codes), lcr / 32, stream, true);
}

extern "C" int trex_tree_split_x3(const float* X, int rows, int cols, int ldx, float max_abs,
                                  void* out, int ldo, void* stream) {
  if (!X || !out || rows <= 0 || cols <= 0 || ldx < cols || ldo < cols || ldo % 4 != 0 ||
      !pos_finite_f32(max_abs) || (reinterpret_cast<uintptr_t>(out) & 15) != 0)
    return set_error(TREX_E_ARG, "trex_tree_split_x3: bad arguments");
  const int64_t n = (int64_t)rows * (ldo / 4);
  hipLaunchKernelGGL(split_x3_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 65536)),
                     dim3(256), 0, (hipStream_t)stream, X, rows, cols, ldx, split_scale(max_abs),
                     static_cast<u32x4*>(out), ldo);
  return tree_hip_check("trex_tree_split_x3");
}

extern "C" int trex_tree_gram_skip_x3p(const void* S16, int N, int64_t K, int skip_rows,
                                       float max_abs, float* G, void* workspace,
                                       int64_t workspace_bytes, void* stream) {
  if (!S16 || !G || !workspace || N <= 0 || K <= 0 || K > 0x7FFFFFFF || skip_rows < 0 ||
      skip_rows > N || !pos_finite_f32(max_abs) || K % 4 != 0)
    return set_error(TREX_E_ARG, "trex_tree_gram_skip_x3p: bad arguments");
  if (workspace_bytes < trex_tree_workspace_bytes(N, K))
    return set_error(TREX_E_ARG, "trex_tree_gram_skip_x3p: workspace too small");
  const float* S = static_cast<const float*>(S16);
  return gram(S, S, N, K, 1, G, static_cast<float*>(workspace), (hipStream_t)stream,
              skip_rows / 64, max_abs, true);
}

// the same Gram with the leaf rows declared exact one-hot by their codes
// (the buffer trex_tree_leaf_codes filled with status 0): their f16 lo plane
// is zero, so the lo x hi products of the leaf strips are skipped, and the
// code rows are read as their bytes instead of 16-B pre-split pieces
// (bitwise the plain call)
extern "C" int trex_tree_gram_skip_x3p_codes(const void* S16, int N, int64_t K, int skip_rows,
                                             float max_abs, const void* codes, int64_t codes_bytes,
                                             int n_leaf, int Q, float* G, void* workspace,
                                             int64_t workspace_bytes, void* stream) {
  if (!S16 || !G || !workspace || N <= 0 || K <= 0 || K > 0x7FFFFFFF || skip_rows < 0 ||
      skip_rows > N || !pos_finite_f32(max_abs) || K % 4 != 0)
    return set_error(TREX_E_ARG, "trex_tree_gram_skip_x3p_codes: bad arguments");
  const int lcr = trex_tree_leaf_code_rows(n_leaf);
  if (!codes || Q != 4 || lcr <= 0 || lcr > N || codes_bytes < (int64_t)lcr * (K / Q))
    return set_error(TREX_E_ARG, "trex_tree_gram_skip_x3p_codes: bad codes (Q = 4, n_leaf >= 32)");
  if (workspace_bytes < trex_tree_workspace_bytes(N, K))
    return set_error(TREX_E_ARG, "trex_tree_gram_skip_x3p_codes: workspace too small");
  const float* S = static_cast<const float*>(S16);
  // TREX_GRAM_LZ (A/B): 0 = every product computed, rows as pre-split f16;
  // 1 = zero-plane products skipped, rows pre-split; default: also the code
  // rows read as their bytes
  const char* ev = std::getenv("TREX_GRAM_LZ");
  const int lz = ev ? std::atoi(ev) : 2;
  const int lzs = lz == 0 ? 0 : lcr / 32;
  return gram(S, S, N, K, 1, G, static_cast<float*>(workspace), (hipStream_t)stream,
              skip_rows / 64, max_abs, true, lzs,
              lz >= 2 ? static_cast<const uint8_t*>(codes) : nullptr);
}

extern "C" int trex_tree_mf_rows_x3p(const void* M16, int ldm, const void* S16, int N, int64_t K,
                                     int row0, int nrows, float max_abs_m, float max_abs_s,
                                     const void* codes, int64_t codes_bytes, int n_leaf, int Q,
                                     float* dS_rows, void* stream) {
  const char* fn = "trex_tree_mf_rows_x3p";
  if (K % 4 != 0 || (codes && Q != 4)) return set_error(TREX_E_ARG, "%s: bad arguments", fn);
  int lcs = 0;
  if (codes) {
    const int lcr = trex_tree_leaf_code_rows(n_leaf);
    if (lcr <= 0 || lcr > N || codes_bytes < (int64_t)lcr * (K / Q))
      return set_error(TREX_E_ARG, "%s: bad codes", fn);
    lcs = lcr / 32;
  }
  return mf_x3(fn, static_cast<const float*>(M16), static_cast<const float*>(S16), N, K, row0,
               nrows, max_abs_m, max_abs_s, dS_rows, static_cast<const uint8_t*>(codes), lcs,
               stream, true, true, ldm);
}

extern "C" int trex_tree_mf(const float* M, const float* S, int N, int64_t K, float* dS,
                            void* stream) {
  return trex_tree_mf_rows(M, S, N, K, 0, N, dS, stream);
}
