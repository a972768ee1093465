// NK landscape-aware loss on MI355X (gfx950): parental logits, the masked
// cross-entropy against the children, and the reverse sweep.
//
// Reference semantics (maraxen/trex):
//   compute_parental_logits               src/trex/evals/benchmark.py:586-663
//   _compute_loss_landscape_aware_stacked src/trex/evals/benchmark.py:235-306
//
// logits[p, i, s] = sum_idx F[i][s * Q^k + idx] * prod_j P[p, nb_j(i), c_j(idx)]
// with idx = sum_j c_j Q^(k-1-j) (neighbour 0 most significant: the
// reference's successive outer products, :637-642, and the (Q, Q^k) reshape of
// the site's table, :647).  k = interactions.shape[1] (padded k, :619).
//
// Layout: sequences S fp32 [N][L][Q] (node-major, the tree path's layout),
// interactions int32 [L][k], fitness fp32 [L][Q^(k+1)].
//
// Kernel mapping (one wave = 64 parent rows of one site): the site's index
// set (its neighbours) and its fitness table are wave-uniform, so the table
// is read with scalar loads and the odometer over the joint index lives in
// SGPRs; each lane gathers its parent's k neighbour distributions into a
// per-lane LDS block [j][c][lane] (conflict-free) and walks the Q^k joint
// states.  The reverse sweep re-walks them: dJ[idx] = sum_s g_s F[s][idx],
// G[j][c_j] += dJ[idx] * prod_{j' != j} P_j'[c_j'] (prefix / suffix products),
// written per (parent, site, j); the combine kernel then sums G over the
// (site, j) pairs that name each neighbour site (inverse-interaction CSR from
// the host plan) -- fixed order, no atomics, bitwise reproducible.  Few
// parents x sites (the reference's eval shape: 31 x 15) take the small-grid
// kernels: a block per (site, 32 parents), the joint states split over 8
// slices of threads and summed in slice order.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "sankoff_dev.h"
#include "trex_common.h"

namespace trex {
namespace {

constexpr int kNkMaxQ = 32;
constexpr int kNkMaxK = 16;
constexpr int32_t kNkMagic = 0x4E4B504C;  // 'NKPL'

int nk_err(const char* fn) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

struct NkArgs {
  const float* S;         // [N][L][Q]
  const int32_t* rows;    // [R] parent rows of S
  const int32_t* inter;   // [L][k]
  const float* F;         // [L][Q^(k+1)]
  int R, L, Q, k, QK;     // QK = Q^k
};

// per-lane LDS block: P_j[c] at ((j * Q + c) * 64 + lane)
__device__ __forceinline__ void gather_neighbours(const NkArgs& a, int row, int site, int lane,
                                                  bool active, float* pl) {
  const cptr<int32_t> inter = as_const(a.inter) + (size_t)site * a.k;
  for (int j = 0; j < a.k; ++j) {
    const int nb = inter[j];
    const float* src = a.S + ((size_t)row * a.L + nb) * a.Q;
    for (int c = 0; c < a.Q; ++c) pl[(j * a.Q + c) * kWave + lane] = active ? src[c] : 0.0f;
  }
}

// The Q^k joint states are walked as (outer, c): outer enumerates the
// digits of neighbours 0..k-2 (an odometer in uniform registers), c the last
// neighbour's state, innermost.  Per outer state the prefix product
// pre = ((f_0 f_1) ... f_{k-2}) -- the association of the reference's
// successive outer products -- is read from the per-lane LDS block (k - 1
// reads), and the inner loop needs only the last neighbour's Q values, which
// stay in registers.  A block holds NS waves that split the outer range
// (parallelism for few parents / large Q^k); partials are combined in a
// fixed wave order.
struct Walk {
  int k, Q, QK, nouter, o0, o1;  // outer states [o0, o1) of this wave
};

__device__ __forceinline__ Walk walk_of(const NkArgs& a, int wave, int ns) {
  Walk w;
  w.k = a.k;
  w.Q = a.Q;
  w.QK = a.QK;
  w.nouter = a.k == 0 ? 1 : a.QK / a.Q;
  const int per = (w.nouter + ns - 1) / ns;
  w.o0 = min(w.nouter, wave * per);
  w.o1 = min(w.nouter, w.o0 + per);
  return w;
}

__device__ __forceinline__ void digits_of(int outer, int k, int Q, int (&d)[kNkMaxK]) {
#pragma unroll
  for (int j = kNkMaxK - 1; j >= 0; --j) {
    if (j < k - 1) {
      d[j] = outer % Q;
      outer /= Q;
    } else {
      d[j] = 0;
    }
  }
}

__device__ __forceinline__ void digits_next(int (&d)[kNkMaxK], int k, int Q) {
  for (int j = k - 2; j >= 0; --j) {
    if (++d[j] < Q) return;
    d[j] = 0;
  }
}

// logits [R][L][Q]; grid (ceil(R/64), L), block (64, NS)
// QT: compile-time Q (2, 4, 20) or 0 = runtime Q <= kNkMaxQ
template <int QT>
__global__ __launch_bounds__(512) void nk_logits_kernel(NkArgs a, float* __restrict__ logits) {
  constexpr int MQ = QT ? QT : kNkMaxQ;
  const int Q = QT ? QT : a.Q;
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int lane = threadIdx.x;
  const int wave = threadIdx.y;
  const int ns = blockDim.y;
  const int site = blockIdx.y;
  const int r = blockIdx.x * kWave + lane;
  const bool active = r < a.R;
  const int row = active ? a.rows[r] : 0;
  float* pl = sh;                                    // [k][Q][64]
  float* part = sh + (size_t)a.k * Q * kWave;      // [NS][Q][64]
  if (wave == 0) gather_neighbours(a, row, site, lane, active, pl);
  __syncthreads();
  const cptr<float> F = as_const(a.F) + (size_t)site * a.QK * Q;
  const Walk w = walk_of(a, wave, ns);
  float last[MQ];  // P_{k-1}[c]
#pragma unroll
  for (int c = 0; c < MQ; ++c)
    last[c] = (a.k > 0 && c < Q) ? pl[((a.k - 1) * Q + c) * kWave + lane] : 1.0f;
  float acc[MQ];
#pragma unroll
  for (int s = 0; s < MQ; ++s) acc[s] = 0.0f;
  int d[kNkMaxK];
  digits_of(w.o0, a.k, Q, d);
  const int inner = a.k == 0 ? 1 : Q;
  for (int outer = w.o0; outer < w.o1; ++outer) {
    float pre = 1.0f;
#pragma unroll
    for (int j = 0; j < kNkMaxK; ++j) {
      if (j < a.k - 1) {
        const float f = pl[(j * Q + d[j]) * kWave + lane];
        pre = j == 0 ? f : pre * f;
      }
    }
    const int base = outer * inner;
#pragma unroll
    for (int c = 0; c < MQ; ++c) {
      if (c < inner) {
        const float p = a.k == 0 ? 1.0f : (a.k == 1 ? last[c] : pre * last[c]);
#pragma unroll
        for (int s = 0; s < MQ; ++s)
          if (s < Q) acc[s] = fmaf(F[(size_t)s * a.QK + base + c], p, acc[s]);
      }
    }
    digits_next(d, a.k, Q);
  }
  if (ns > 1) {
    for (int s = 0; s < Q; ++s) part[((size_t)wave * Q + s) * kWave + lane] = acc[s];
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int s = 0; s < MQ; ++s) {
      if (s < Q) {
        float v = part[(size_t)s * kWave + lane];
        for (int y = 1; y < ns; ++y) v += part[((size_t)y * Q + s) * kWave + lane];
        acc[s] = v;
      }
    }
  }
  if (active) {
    float* o = logits + ((size_t)r * a.L + site) * Q;
#pragma unroll
    for (int s = 0; s < MQ; ++s)
      if (s < Q) o[s] = acc[s];
  }
}

// reverse: G [R][L][k][Q] = d(sum g * logits)/d P_j  (per site, per slot j).
// Per outer state: E_j = prod_{j' < k-1, j' != j} f_j' (prefix x suffix),
// inner c: dJ_c = sum_s g_s F[s][outer*Q + c]; G[k-1][c] += dJ_c * pre (in
// registers); T = sum_c dJ_c P_{k-1}[c]; then G[j][d_j] += E_j * T (LDS).
template <int QT>
__global__ __launch_bounds__(512) void nk_logits_bwd_kernel(NkArgs a, const float* __restrict__ g,
                                                            float* __restrict__ G) {
  constexpr int MQ = QT ? QT : kNkMaxQ;
  const int Q = QT ? QT : a.Q;
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int lane = threadIdx.x;
  const int wave = threadIdx.y;
  const int ns = blockDim.y;
  const int site = blockIdx.y;
  const int r = blockIdx.x * kWave + lane;
  const bool active = r < a.R;
  const int row = active ? a.rows[r] : 0;
  const int kq = a.k * Q;
  float* pl = sh;                                          // [k][Q][64]
  float* gl = sh + (size_t)kq * kWave * (1 + wave);        // this wave's bins [k][Q][64]
  if (wave == 0) gather_neighbours(a, row, site, lane, active, pl);
  for (int t = 0; t < kq; ++t) gl[t * kWave + lane] = 0.0f;
  __syncthreads();
  float gs[MQ];
  const float* gp = g + ((size_t)(active ? r : 0) * a.L + site) * Q;
#pragma unroll
  for (int s = 0; s < MQ; ++s) gs[s] = (s < Q && active) ? gp[s] : 0.0f;
  const cptr<float> F = as_const(a.F) + (size_t)site * a.QK * Q;
  const Walk w = walk_of(a, wave, ns);
  float last[MQ], glast[MQ];
#pragma unroll
  for (int c = 0; c < MQ; ++c) {
    last[c] = c < Q ? pl[((a.k - 1) * Q + c) * kWave + lane] : 0.0f;
    glast[c] = 0.0f;
  }
  int d[kNkMaxK];
  digits_of(w.o0, a.k, Q, d);
  for (int outer = w.o0; outer < w.o1; ++outer) {
    float f[kNkMaxK], E[kNkMaxK];
#pragma unroll
    for (int j = 0; j < kNkMaxK; ++j) f[j] = j < a.k - 1 ? pl[(j * Q + d[j]) * kWave + lane] : 1.0f;
    float pre = 1.0f;
#pragma unroll
    for (int j = 0; j < kNkMaxK; ++j) {
      E[j] = pre;
      pre *= f[j];
    }
    float suf = 1.0f;
#pragma unroll
    for (int j = kNkMaxK - 1; j >= 0; --j) {
      E[j] *= suf;
      suf *= f[j];
    }
    const int base = outer * Q;
    float T = 0.0f;
#pragma unroll
    for (int c = 0; c < MQ; ++c) {
      if (c < Q) {
        float dj = 0.0f;
#pragma unroll
        for (int s = 0; s < MQ; ++s)
          if (s < Q) dj = fmaf(gs[s], F[(size_t)s * a.QK + base + c], dj);
        glast[c] = fmaf(dj, pre, glast[c]);
        T = fmaf(dj, last[c], T);
      }
    }
#pragma unroll
    for (int j = 0; j < kNkMaxK; ++j)
      if (j < a.k - 1) {
        float* gg = gl + (j * Q + d[j]) * kWave + lane;
        *gg = fmaf(E[j], T, *gg);
      }
    digits_next(d, a.k, Q);
  }
  for (int c = 0; c < Q; ++c) gl[((a.k - 1) * Q + c) * kWave + lane] = glast[c];
  __syncthreads();
  if (wave != 0 || !active) return;
  float* o = G + (((size_t)r * a.L + site) * a.k) * Q;
  for (int t = 0; t < kq; ++t) {
    float v = sh[(size_t)kq * kWave + t * kWave + lane];
    for (int y = 1; y < ns; ++y) v += sh[(size_t)kq * kWave * (1 + y) + t * kWave + lane];
    o[t] = v;
  }
}

// ---- small grids (the reference's eval shape: 32 parents x 15 sites, Q = 2,
// k = 10: 15 one-wave-per-64-parents blocks, each walking 512 joint states
// serially, 49 + 78 us) -------------------------------------------------------
// A block = one site x kNkSmallP parents x kNkSlices slices of the joint index:
// thread (slice, parent) walks a contiguous range of idx with an odometer,
// the site's fitness table and the parents' neighbour distributions in LDS;
// the slices' partial sums combine in fixed slice order.  Same products
// (left to right over the neighbours, the reference's successive outer
// products) and prefix / suffix gradients as the kernels above.
// masked cross-entropy of every child of parent pc at site l against
// log_softmax of the parent's logits xv (benchmark.py:288-302): d logits,
// d child rows, the (pc, l) partial of the loss
struct NkCe {
  const float* S;
  const int32_t* cofs;
  const int32_t* cidx;
  const float* mask;
  float scale;
  float* dlog;
  float* dchild;
  double* part;
};
__device__ __forceinline__ void nk_ce_one(const NkCe& c, const float (&xv)[kNkMaxQ], int pc, int l,
                                          int L, int Q) {
  const size_t t = (size_t)pc * L + l;
  float mx = -INFINITY;
#pragma unroll
  for (int s = 0; s < kNkMaxQ; ++s) mx = fmaxf(mx, xv[s]);
  float se = 0.0f;
#pragma unroll
  for (int s = 0; s < kNkMaxQ; ++s)
    if (s < Q) se += expf(xv[s] - mx);
  const float lse = mx + logf(se);
  const float mk = c.mask ? c.mask[l] : 1.0f;
  float dl[kNkMaxQ];
#pragma unroll
  for (int s = 0; s < kNkMaxQ; ++s) dl[s] = 0.0f;
  double ce = 0.0;
  for (int e = c.cofs[pc]; e < c.cofs[pc + 1]; ++e) {
    const int n = c.cidx[e];
    const float* sn = c.S + ((size_t)n * L + l) * Q;
    float* dc = c.dchild + ((size_t)n * L + l) * Q;
    float tot = 0.0f, cen = 0.0f;
#pragma unroll
    for (int s = 0; s < kNkMaxQ; ++s)
      if (s < Q) {
        const float v = sn[s];
        const float lp = xv[s] - lse;
        tot += v;
        cen -= v * lp;
        dc[s] = -c.scale * mk * lp;
        dl[s] -= v;
      }
#pragma unroll
    for (int s = 0; s < kNkMaxQ; ++s)
      if (s < Q) dl[s] += expf(xv[s] - lse) * tot;
    ce += (double)(mk * cen);
  }
  float* dlo = c.dlog + t * Q;
#pragma unroll
  for (int s = 0; s < kNkMaxQ; ++s)
    if (s < Q) dlo[s] = c.scale * mk * dl[s];
  c.part[t] = ce;
}

// ---- few (parent, site) pairs (the reference's eval shape: 31 x 15, Q = 2,
// K = 10): one workgroup per pair, its threads over the Q^k joint states.
// The wave-per-64-parents kernels above walk every joint state serially per
// lane (serial chains of dependent table reads: 49 / 78 us for 2 M MACs);
// here each thread takes joint states t, t + 256, ...: the product over the
// k neighbours left to right (the reference's successive outer products),
// F[s][idx] times it, and the block sums its threads in a fixed tree order.
constexpr int kNkPP = 256;  // threads per (parent, site) workgroup

// digits of idx, neighbour 0 most significant (Q = 2: shifts)
template <int QT>
__device__ __forceinline__ int nk_digit(int idx, int j, int k, int Q) {
  if constexpr (QT == 2) return (idx >> (k - 1 - j)) & 1;
  int v = idx;
  for (int t = k - 1; t > j; --t) v /= Q;
  return v % Q;
}

// fixed-order block sum of n values per thread (LDS red[n][kNkPP]); thread 0
// gets the totals in out
template <int NV>
__device__ __forceinline__ void nk_block_sum(float (&v)[NV], int n, float* red) {
  const int t = threadIdx.x;
  for (int q = 0; q < n; ++q) red[q * kNkPP + t] = v[q];
  __syncthreads();
  for (int w = kNkPP / 2; w > 0; w >>= 1) {
    if (t < w)
      for (int q = 0; q < n; ++q) red[q * kNkPP + t] += red[q * kNkPP + t + w];
    __syncthreads();
  }
  for (int q = 0; q < n; ++q) v[q] = red[q * kNkPP];
}

// the parent's k neighbour distributions at this site, P[j][c], into LDS
__device__ __forceinline__ void nk_pp_stage(const NkArgs& a, int r, int site, float* P) {
  const int32_t* inter = a.inter + (size_t)site * a.k;
  for (int e = threadIdx.x; e < a.k * a.Q; e += kNkPP) {
    const int j = e / a.Q, c = e - j * a.Q;
    P[e] = a.S[((size_t)a.rows[r] * a.L + inter[j]) * a.Q + c];
  }
}

template <int QT, bool CE>
__global__ __launch_bounds__(kNkPP) void nk_logits_pp_kernel(NkArgs a, float* __restrict__ logits,
                                                              NkCe ce) {
  constexpr int MQ = QT ? QT : kNkMaxQ;
  const int Q = QT ? QT : a.Q, k = a.k, QK = a.QK;
  __shared__ float P[kNkMaxK * kNkMaxQ];
  __shared__ float red[MQ * kNkPP];
  const int site = blockIdx.x % a.L, r = blockIdx.x / a.L;
  nk_pp_stage(a, r, site, P);
  __syncthreads();
  const float* F = a.F + (size_t)site * QK * Q;
  float acc[MQ];
#pragma unroll
  for (int s = 0; s < MQ; ++s) acc[s] = 0.0f;
  for (int idx = threadIdx.x; idx < QK; idx += kNkPP) {
    float prod = k > 0 ? P[nk_digit<QT>(idx, 0, k, Q)] : 1.0f;
    for (int j = 1; j < k; ++j) prod = prod * P[j * Q + nk_digit<QT>(idx, j, k, Q)];
#pragma unroll
    for (int s = 0; s < MQ; ++s)
      if (s < Q) acc[s] = fmaf(F[(size_t)s * QK + idx], prod, acc[s]);
  }
  nk_block_sum<MQ>(acc, Q, red);
  if (threadIdx.x != 0) return;
  if constexpr (CE) {
    float xv[kNkMaxQ];
#pragma unroll
    for (int s = 0; s < kNkMaxQ; ++s) xv[s] = s < Q ? acc[s < MQ ? s : 0] : -INFINITY;
    nk_ce_one(ce, xv, r, site, a.L, Q);
  } else {
    for (int s = 0; s < Q; ++s) logits[((size_t)r * a.L + site) * Q + s] = acc[s];
  }
}

// reverse: w(idx) = sum_s g_s F[s][idx]; bin (j, c_j(idx)) += w * prod_{j' != j}
// P[j'][c_j'] (prefix x suffix products), per-thread bins summed in a fixed
// tree order; G[r][site][j][c]
template <int QT>
__global__ __launch_bounds__(kNkPP) void nk_logits_bwd_pp_kernel(NkArgs a,
                                                                  const float* __restrict__ g,
                                                                  float* __restrict__ G) {
  constexpr int MQ = QT ? QT : kNkMaxQ;
  constexpr int MB = QT ? kNkMaxK * QT : kNkMaxK * kNkMaxQ;  // bins per thread
  const int Q = QT ? QT : a.Q, k = a.k, QK = a.QK;
  __shared__ float P[kNkMaxK * kNkMaxQ];
  extern __shared__ float redb[];  // [k * Q][kNkPP]
  const int site = blockIdx.x % a.L, r = blockIdx.x / a.L;
  nk_pp_stage(a, r, site, P);
  __syncthreads();
  const float* F = a.F + (size_t)site * QK * Q;
  float gs[MQ];
#pragma unroll
  for (int s = 0; s < MQ; ++s) gs[s] = s < Q ? g[((size_t)r * a.L + site) * Q + s] : 0.0f;
  float bins[MB];
#pragma unroll
  for (int b = 0; b < MB; ++b) bins[b] = 0.0f;
  for (int idx = threadIdx.x; idx < QK; idx += kNkPP) {
    float w = 0.0f;
#pragma unroll
    for (int s = 0; s < MQ; ++s)
      if (s < Q) w = fmaf(gs[s], F[(size_t)s * QK + idx], w);
    int c[kNkMaxK];
    float pre[kNkMaxK];
    float acc = 1.0f;
#pragma unroll
    for (int j = 0; j < kNkMaxK; ++j) {
      if (j < k) {
        c[j] = nk_digit<QT>(idx, j, k, Q);
        pre[j] = acc;
        acc = acc * P[j * Q + c[j]];
      }
    }
    float suf = 1.0f;
#pragma unroll
    for (int j = kNkMaxK - 1; j >= 0; --j) {
      if (j < k) {
        const float v = w * (pre[j] * suf);
#pragma unroll
        for (int q = 0; q < MQ; ++q)
          if (q == c[j]) bins[j * MQ + q] += v;
        suf = suf * P[j * Q + c[j]];
      }
    }
  }
  // fixed-order tree sum of the k * Q bins over the threads
  const int t = threadIdx.x;
  const int nbin = k * Q;
  for (int j = 0; j < k; ++j)
    for (int q = 0; q < Q; ++q) redb[(j * Q + q) * kNkPP + t] = bins[j * MQ + (q < MQ ? q : 0)];
  __syncthreads();
  for (int w = kNkPP / 2; w > 0; w >>= 1) {
    if (t < w)
      for (int b = 0; b < nbin; ++b) redb[b * kNkPP + t] += redb[b * kNkPP + t + w];
    __syncthreads();
  }
  for (int b = t; b < nbin; b += kNkPP) G[((size_t)r * a.L + site) * nbin + b] = redb[b * kNkPP];
}

// ---- register kernels for small joint spaces (Q = 4, k <= 4; Q = 2,
// k <= 6; the DNA shape, 255 parents x 2 000 sites, Q 4, k 4) ------------------
// The wave-per-64-parents kernels above take each lane's prefix factors from
// its LDS block and wait on a scalar load chain per F value (≈10 % of the
// VALU peak).  Here Q and k are compile-time and a lane holds PPL parents'
// k neighbour distributions in VGPRs.  The digits of neighbours 0..k-3 run
// as nested rolled loops (each rotates its neighbour's Q factors -- and in
// the reverse its Q bins -- by one register after every iteration, so the
// current digit's value always sits in slot 0: no indexed register access)
// around an unrolled body over neighbour k-2's digit and the last
// neighbour's state; each body issues its 4 Q^2 F values as wide scalar
// loads, and every F value feeds PPL parents.  The arithmetic per (parent,
// site) is the rolled kernel's at NS = 1 step for step (the same products,
// fmas and their order): the results are bitwise equal to it.
constexpr int nk_cpow(int b, int e) { return e <= 0 ? 1 : b * nk_cpow(b, e - 1); }

constexpr int kNkRegSites = 4;  // sites (waves) per block

template <int Q>
__device__ __forceinline__ void nk_rot(float (&v)[Q]) {
  const float t = v[0];
#pragma unroll
  for (int c = 0; c < Q - 1; ++c) v[c] = v[c + 1];
  v[Q - 1] = t;
}

template <int Q, int K, int PPL>
__device__ __forceinline__ void nk_reg_gather(const NkArgs& a, int site, int lane,
                                              float (&f)[PPL][K][Q], int (&rr)[PPL]) {
  const cptr<int32_t> inter = as_const(a.inter) + (size_t)site * K;
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    const int r = (blockIdx.x * PPL + p) * kWave + lane;
    rr[p] = r < a.R ? r : -1;
    const int row = r < a.R ? a.rows[r] : 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const float* src = a.S + ((size_t)row * a.L + inter[j]) * Q;
      if constexpr (Q == 4) {
        const float4 v = r < a.R ? *reinterpret_cast<const float4*>(src) : make_float4(0, 0, 0, 0);
        f[p][j][0] = v.x;
        f[p][j][1] = v.y;
        f[p][j][2] = v.z;
        f[p][j][3] = v.w;
      } else {
        const float2 v = r < a.R ? *reinterpret_cast<const float2*>(src) : make_float2(0, 0);
        f[p][j][0] = v.x;
        f[p][j][1] = v.y;
      }
    }
  }
}

// forward body: the Q outer states of one setting of the rolled digits
// (their factors in slot 0 of f[p][0..k-3]); F at this body's first entry
template <int Q, int K, int PPL>
__device__ __forceinline__ void nk_fwd_body(const float (&f)[PPL][K][Q], cptr<float> F,
                                            float (&acc)[PPL][Q]) {
  constexpr int QK = nk_cpow(Q, K);
  constexpr int NI = K >= 2 ? Q : 1;
  float ph[PPL];  // ((f_0 f_1) ...) f_{k-3}
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    ph[p] = 1.0f;
#pragma unroll
    for (int j = 0; j < K - 2; ++j) ph[p] = j == 0 ? f[p][j][0] : ph[p] * f[p][j][0];
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
#pragma unroll
    for (int c = 0; c < Q; ++c) {
#pragma unroll
      for (int p = 0; p < PPL; ++p) {
        float pv;
        if constexpr (K == 1)
          pv = f[p][0][c];
        else if constexpr (K == 2)
          pv = f[p][0][i] * f[p][1][c];
        else
          pv = (ph[p] * f[p][K - 2][i]) * f[p][K - 1][c];
#pragma unroll
        for (int s = 0; s < Q; ++s) acc[p][s] = fmaf(F[s * QK + i * Q + c], pv, acc[p][s]);
      }
    }
  }
}

// rolled digit J (J < k - 2): Q iterations, neighbour J's factors rotated
template <int Q, int K, int PPL, int J>
__device__ __forceinline__ void nk_fwd_loop(float (&f)[PPL][K][Q], cptr<float> F,
                                            float (&acc)[PPL][Q]) {
  if constexpr (J >= K - 2) {
    nk_fwd_body<Q, K, PPL>(f, F, acc);
  } else {
    constexpr int step = nk_cpow(Q, K - 1 - J);  // F entries per digit-J value
#pragma unroll 1
    for (int d = 0; d < Q; ++d) {
      nk_fwd_loop<Q, K, PPL, J + 1>(f, F + d * step, acc);
#pragma unroll
      for (int p = 0; p < PPL; ++p) nk_rot<Q>(f[p][J]);
    }
  }
}

template <int Q, int K, int PPL>
__global__ __launch_bounds__(kWave * kNkRegSites) __attribute__((amdgpu_waves_per_eu(4))) void nk_logits_reg_kernel(NkArgs a,
                                                                            float* __restrict__ logits) {
  constexpr int QK = nk_cpow(Q, K);
  const int site = __builtin_amdgcn_readfirstlane(blockIdx.y * kNkRegSites + threadIdx.y);
  if (site >= a.L) return;
  const int lane = threadIdx.x;
  float f[PPL][K][Q];
  int rr[PPL];
  nk_reg_gather<Q, K, PPL>(a, site, lane, f, rr);
  float acc[PPL][Q];
#pragma unroll
  for (int p = 0; p < PPL; ++p)
#pragma unroll
    for (int s = 0; s < Q; ++s) acc[p][s] = 0.0f;
  nk_fwd_loop<Q, K, PPL, 0>(f, as_const(a.F) + (size_t)site * QK * Q, acc);
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    if (rr[p] < 0) continue;
    float* o = logits + ((size_t)rr[p] * a.L + site) * Q;
    if constexpr (Q == 4)
      *reinterpret_cast<float4*>(o) = make_float4(acc[p][0], acc[p][1], acc[p][2], acc[p][3]);
    else
      *reinterpret_cast<float2*>(o) = make_float2(acc[p][0], acc[p][1]);
  }
}

// reverse body: the rolled nk_logits_bwd_kernel's per-outer-state steps
// (prefix x suffix products E_j, dJ_c, the last neighbour's bins, T, the
// other neighbours' bins) for the Q outer states of one rolled setting;
// neighbour j < k-2's current factor and bin sit in slot 0
template <int Q, int K, int PPL>
__device__ __forceinline__ void nk_bwd_body(const float (&f)[PPL][K][Q], const float (&gs)[PPL][Q],
                                            cptr<float> F, float (&gb)[PPL][K][Q]) {
  constexpr int QK = nk_cpow(Q, K);
  constexpr int NI = K >= 2 ? Q : 1;
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      float fv[K], E[K];
#pragma unroll
      for (int j = 0; j < K; ++j)
        fv[j] = j < K - 2 ? f[p][j][0] : (j == K - 2 ? f[p][j][i] : 1.0f);
      float pre = 1.0f;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        E[j] = pre;
        pre *= fv[j];
      }
      float suf = 1.0f;
#pragma unroll
      for (int j = K - 1; j >= 0; --j) {
        E[j] *= suf;
        suf *= fv[j];
      }
      float T = 0.0f;
#pragma unroll
      for (int c = 0; c < Q; ++c) {
        float dj = 0.0f;
#pragma unroll
        for (int s = 0; s < Q; ++s) dj = fmaf(gs[p][s], F[s * QK + i * Q + c], dj);
        gb[p][K - 1][c] = fmaf(dj, pre, gb[p][K - 1][c]);
        T = fmaf(dj, f[p][K - 1][c], T);
      }
#pragma unroll
      for (int j = 0; j < K - 1; ++j) {
        const int d = j < K - 2 ? 0 : i;
        gb[p][j][d] = fmaf(E[j], T, gb[p][j][d]);
      }
    }
  }
}

template <int Q, int K, int PPL, int J>
__device__ __forceinline__ void nk_bwd_loop(float (&f)[PPL][K][Q], const float (&gs)[PPL][Q],
                                            cptr<float> F, float (&gb)[PPL][K][Q]) {
  if constexpr (J >= K - 2) {
    nk_bwd_body<Q, K, PPL>(f, gs, F, gb);
  } else {
    constexpr int step = nk_cpow(Q, K - 1 - J);
#pragma unroll 1
    for (int d = 0; d < Q; ++d) {
      nk_bwd_loop<Q, K, PPL, J + 1>(f, gs, F + d * step, gb);
#pragma unroll
      for (int p = 0; p < PPL; ++p) {
        nk_rot<Q>(f[p][J]);
        nk_rot<Q>(gb[p][J]);
      }
    }
  }
}

template <int Q, int K, int PPL>
__global__ __launch_bounds__(kWave * kNkRegSites) void nk_logits_bwd_reg_kernel(
    NkArgs a, const float* __restrict__ g, float* __restrict__ G) {
  constexpr int QK = nk_cpow(Q, K);
  const int site = __builtin_amdgcn_readfirstlane(blockIdx.y * kNkRegSites + threadIdx.y);
  if (site >= a.L) return;
  const int lane = threadIdx.x;
  float f[PPL][K][Q];
  int rr[PPL];
  nk_reg_gather<Q, K, PPL>(a, site, lane, f, rr);
  float gs[PPL][Q], gb[PPL][K][Q];
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    const float* gp = g + ((size_t)(rr[p] < 0 ? 0 : rr[p]) * a.L + site) * Q;
#pragma unroll
    for (int s = 0; s < Q; ++s) gs[p][s] = rr[p] < 0 ? 0.0f : gp[s];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int c = 0; c < Q; ++c) gb[p][j][c] = 0.0f;
  }
  nk_bwd_loop<Q, K, PPL, 0>(f, gs, as_const(a.F) + (size_t)site * QK * Q, gb);
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    if (rr[p] < 0) continue;
    float* o = G + (((size_t)rr[p] * a.L + site) * K) * Q;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if constexpr (Q == 4)
        *reinterpret_cast<float4*>(o + j * Q) = make_float4(gb[p][j][0], gb[p][j][1], gb[p][j][2], gb[p][j][3]);
      else
        *reinterpret_cast<float2*>(o + j * Q) = make_float2(gb[p][j][0], gb[p][j][1]);
    }
  }
}

// the register kernels take (Q, k) with Q^(k-1) <= 64 at Q = 4 or 2
bool nk_use_reg(int Q, int k) {
  const char* e = std::getenv("TREX_NK_REG");  // A/B: "0" keeps the rolled kernels (read per call)
  if (e && e[0] == '0') return false;
  return (Q == 4 && k >= 1 && k <= 4) || (Q == 2 && k >= 1 && k <= 6);
}

constexpr int kNkRegPplFwd = 2, kNkRegPplBwd = 2;

template <int Q, int K>
void nk_reg_launch(const NkArgs& a, hipStream_t st, float* logits, const float* g, float* G) {
  const int ppl = logits ? kNkRegPplFwd : kNkRegPplBwd;
  const dim3 grid((a.R + kWave * ppl - 1) / (kWave * ppl), (a.L + kNkRegSites - 1) / kNkRegSites);
  const dim3 block(kWave, kNkRegSites);
  if (logits)
    hipLaunchKernelGGL((nk_logits_reg_kernel<Q, K, kNkRegPplFwd>), grid, block, 0, st, a, logits);
  else
    hipLaunchKernelGGL((nk_logits_bwd_reg_kernel<Q, K, kNkRegPplBwd>), grid, block, 0, st, a, g, G);
}

// logits (g, G null) or their reverse (logits null)
void nk_reg_run(const NkArgs& a, hipStream_t st, float* logits, const float* g, float* G) {
  if (a.Q == 4) {
    switch (a.k) {
      case 1: nk_reg_launch<4, 1>(a, st, logits, g, G); break;
      case 2: nk_reg_launch<4, 2>(a, st, logits, g, G); break;
      case 3: nk_reg_launch<4, 3>(a, st, logits, g, G); break;
      default: nk_reg_launch<4, 4>(a, st, logits, g, G); break;
    }
  } else {
    switch (a.k) {
      case 1: nk_reg_launch<2, 1>(a, st, logits, g, G); break;
      case 2: nk_reg_launch<2, 2>(a, st, logits, g, G); break;
      case 3: nk_reg_launch<2, 3>(a, st, logits, g, G); break;
      case 4: nk_reg_launch<2, 4>(a, st, logits, g, G); break;
      case 5: nk_reg_launch<2, 5>(a, st, logits, g, G); break;
      default: nk_reg_launch<2, 6>(a, st, logits, g, G); break;
    }
  }
}

// the per-pair kernels for few (parent, site) pairs with many joint states
bool nk_use_pp(int R, int L, int Q, int k, int QK) {
  if (k == 0 || (Q != 2 && Q != 4)) return false;
  static const int force = [] {  // A/B: TREX_NK_PP=1 at any R * L
    const char* e = std::getenv("TREX_NK_PP");
    return e ? std::atoi(e) : -1;
  }();
  if (force == 0) return false;
  return ((int64_t)R * L <= 4096 || force == 1) && QK >= kNkPP;
}


// Cross-entropy of every child against its parent's logits (benchmark.py
// :292-300).  One lane per (compact parent pc, site).  Writes
//   dlog[pc][l][:]  = scale * mask_l * sum_children (softmax * sum_s S_n - S_n)
//   dchild[n][l][:] = -scale * mask_l * log_softmax(logits[pc(n)])
//   part[pc * L + l] = sum_children -mask_l * sum_s S_n * logp   (fp64)
__global__ __launch_bounds__(256) void nk_ce_kernel(const float* __restrict__ S,
                                                    const float* __restrict__ logits,
                                                    const int32_t* __restrict__ cofs,
                                                    const int32_t* __restrict__ cidx,
                                                    const float* __restrict__ mask, int nP, int L,
                                                    int Q, float scale, float* __restrict__ dlog,
                                                    float* __restrict__ dchild,
                                                    double* __restrict__ part) {
  const NkCe ce{S, cofs, cidx, mask, scale, dlog, dchild, part};
  const int64_t total = (int64_t)nP * L;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const float* x = logits + (size_t)t * Q;
    float xv[kNkMaxQ];
#pragma unroll
    for (int s = 0; s < kNkMaxQ; ++s) xv[s] = s < Q ? x[s] : -INFINITY;
    nk_ce_one(ce, xv, (int)(t / L), (int)(t % L), L, Q);
  }
}

// Q = 4: the same cross-entropy with one 16-B access per row (float4 logits,
// child rows, d child, d logits) instead of four strided dwords -- the
// arithmetic of nk_ce_one step for step (bitwise the generic kernel)
__global__ __launch_bounds__(256) void nk_ce4_kernel(const float4* __restrict__ S,
                                                     const float4* __restrict__ logits,
                                                     const int32_t* __restrict__ cofs,
                                                     const int32_t* __restrict__ cidx,
                                                     const float* __restrict__ mask, int nP, int L,
                                                     float scale, float4* __restrict__ dlog,
                                                     float4* __restrict__ dchild,
                                                     double* __restrict__ part) {
  const int64_t total = (int64_t)nP * L;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int pc = (int)(t / L), l = (int)(t - (int64_t)pc * L);
    const float4 x4 = logits[t];
    const float xv[4] = {x4.x, x4.y, x4.z, x4.w};
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < 4; ++s) mx = fmaxf(mx, xv[s]);
    float se = 0.0f;
#pragma unroll
    for (int s = 0; s < 4; ++s) se += expf(xv[s] - mx);
    const float lse = mx + logf(se);
    const float mk = mask ? mask[l] : 1.0f;
    float dl[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    double ce = 0.0;
    for (int e = cofs[pc]; e < cofs[pc + 1]; ++e) {
      const size_t row = (size_t)cidx[e] * L + l;
      const float4 v4 = S[row];
      const float sv[4] = {v4.x, v4.y, v4.z, v4.w};
      float tot = 0.0f, cen = 0.0f, dcv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float lp = xv[s] - lse;
        tot += sv[s];
        cen -= sv[s] * lp;
        dcv[s] = -scale * mk * lp;
        dl[s] -= sv[s];
      }
      dchild[row] = make_float4(dcv[0], dcv[1], dcv[2], dcv[3]);
#pragma unroll
      for (int s = 0; s < 4; ++s) dl[s] += expf(xv[s] - lse) * tot;
      ce += (double)(mk * cen);
    }
    dlog[t] = make_float4(scale * mk * dl[0], scale * mk * dl[1], scale * mk * dl[2],
                          scale * mk * dl[3]);
    part[t] = ce;
  }
}

// fixed-order two-level sum of the CE partials: block b sums chunk b into
// sums[b]; nk_loss_kernel then sums the chunks and writes
// loss = surrogate + lambda * ce / norm
constexpr int kNkChunks = 256;
constexpr int64_t kNkDirectParts = 8192;
__global__ __launch_bounds__(256) void nk_chunk_sum_kernel(const double* __restrict__ part,
                                                           int64_t n, double* __restrict__ sums) {
  __shared__ double red[256];
  const int64_t per = (n + kNkChunks - 1) / kNkChunks;
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = min(n, lo + per);
  double v = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) v += part[i];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void nk_loss_kernel(const double* __restrict__ part, int64_t n,
                                                      const float* __restrict__ surrogate,
                                                      double coef, float* __restrict__ loss) {
  __shared__ double red[256];
  double v = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) v += part[i];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = (float)((surrogate ? (double)surrogate[0] : 0.0) + coef * red[0]);
}

// d_seqs = d_seqs_in + dchild + (for a parent row) the gathered per-slot
// logits gradients: for site m of parent pc, the sum over the inverse-
// interaction entries of m of G[pc][site][j][q] (trex_nk_plan_build order)
__global__ __launch_bounds__(256) void nk_combine_kernel(const float* __restrict__ din,
                                                         const float* __restrict__ dchild,
                                                         const float* __restrict__ G,
                                                         const int32_t* __restrict__ iofs,
                                                         const int32_t* __restrict__ ient,
                                                         const int32_t* __restrict__ rowmap,
                                                         int N, int L, int Q, int k,
                                                         float* __restrict__ dout) {
  const int64_t per = (int64_t)L * Q;
  const int64_t total = (int64_t)N * per;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(t / per);
    const int64_t w = t - (int64_t)n * per;
    const int pc = rowmap[n];
    float v = (din ? din[t] : 0.0f) + dchild[t];
    if (pc >= 0) {
      float acc = 0.0f;
      if (G) {
        const int m = (int)(w / Q), q = (int)(w - (int64_t)m * Q);
        for (int e = iofs[m]; e < iofs[m + 1]; ++e)
          acc += G[((size_t)pc * L * k + ient[e]) * Q + q];
      }
      v += acc;
    }
    dout[t] = v;
  }
}

// Q = 4: one thread per (node, site) row, float4 rows and gathers (the
// generic kernel's per-state sums in the same order: bitwise)
__global__ __launch_bounds__(256) void nk_combine4_kernel(const float4* __restrict__ din,
                                                          const float4* __restrict__ dchild,
                                                          const float4* __restrict__ G,
                                                          const int32_t* __restrict__ iofs,
                                                          const int32_t* __restrict__ ient,
                                                          const int32_t* __restrict__ rowmap,
                                                          int N, int L, int k,
                                                          float4* __restrict__ dout) {
  const int64_t total = (int64_t)N * L;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(t / L), m = (int)(t - (int64_t)n * L);
    const int pc = rowmap[n];
    const float4 a = din ? din[t] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const float4 b = dchild[t];
    float4 v = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    if (pc >= 0 && G) {
      float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      for (int e = iofs[m]; e < iofs[m + 1]; ++e) {
        const float4 gv = G[(size_t)pc * L * k + ient[e]];
        acc.x += gv.x;
        acc.y += gv.y;
        acc.z += gv.z;
        acc.w += gv.w;
      }
      v.x += acc.x;
      v.y += acc.y;
      v.z += acc.z;
      v.w += acc.w;
    }
    dout[t] = v;
  }
}

// Q = 4, one workgroup per node row n when the parent row's per-slot
// gradients G [L][k] (16 B each) fit the LDS: the block is staged with
// coalesced 16-B loads and the inverse-CSR gathers read LDS (each 16-B
// gather from L2 pulled a whole 128-B line: 8x the bytes, 40 us at the DNA
// shape); sums in nk_combine4_kernel's order (bitwise the same)
constexpr int kNkCombineThreads = 1024;
constexpr int64_t kNkCombineLds = 160 * 1024;
inline bool misaligned16(const void* p) { return p && (reinterpret_cast<uintptr_t>(p) & 15u); }
__global__ __launch_bounds__(kNkCombineThreads) void nk_combine4_lds_kernel(
    const float4* __restrict__ din, const float4* __restrict__ dchild,
    const float4* __restrict__ G, const int32_t* __restrict__ iofs,
    const int32_t* __restrict__ ient, const int32_t* __restrict__ rowmap, int L, int k,
    float4* __restrict__ dout) {
  extern __shared__ __attribute__((aligned(16))) float4 gl[];
  const int n = blockIdx.x;
  const int pc = rowmap[n];
  const size_t rb = (size_t)n * L;
  if (pc >= 0) {  // block-uniform
    const float4* gp = G + (size_t)pc * L * k;
    for (int e = threadIdx.x; e < L * k; e += kNkCombineThreads) gl[e] = gp[e];
    __syncthreads();
  }
  for (int m = threadIdx.x; m < L; m += kNkCombineThreads) {
    const float4 a = din ? din[rb + m] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const float4 b = dchild[rb + m];
    float4 v = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    if (pc >= 0) {
      float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      for (int e = iofs[m]; e < iofs[m + 1]; ++e) {
        const float4 gv = gl[ient[e]];
        acc.x += gv.x;
        acc.y += gv.y;
        acc.z += gv.z;
        acc.w += gv.w;
      }
      v.x += acc.x;
      v.y += acc.y;
      v.z += acc.z;
      v.w += acc.w;
    }
    dout[rb + m] = v;
  }
}

int64_t ipow(int b, int e) {
  int64_t r = 1;
  for (int i = 0; i < e; ++i) r *= b;
  return r;
}

int nk_check(const char* fn, int L, int Q, int k) {
  if (L <= 0 || Q < 2 || Q > kNkMaxQ || k < 0 || k > kNkMaxK)
    return set_error(TREX_E_ARG, "%s: bad shape L=%d Q=%d k=%d (Q <= %d, k <= %d)", fn, L, Q, k,
                     kNkMaxQ, kNkMaxK);
  if (k * Q > 128)  // per-lane LDS blocks: 2 * k * Q * 64 * 4 B <= 64 KiB
    return set_error(TREX_E_UNSUPPORTED, "%s: k * Q = %d > 128 not supported", fn, k * Q);
  if (ipow(Q, k + 1) > (1LL << 26))
    return set_error(TREX_E_UNSUPPORTED, "%s: fitness table Q^(k+1) too large", fn);
  return TREX_OK;
}

// waves per block splitting the outer joint states: enough waves to fill
// the chip when there are few (parent-group, site) blocks, each wave with
// >= 2 outer states, and the bwd's per-wave LDS bins within 64 KiB
int nk_slices(int R, int L, int Q, int k) {
  if (k == 0) return 1;
  const int64_t nouter = ipow(Q, k - 1);
  const int64_t blocks = (int64_t)((R + kWave - 1) / kWave) * L;
  int ns = 1;
  while (ns < 8 && blocks * ns < 4096 && nouter >= 4LL * ns &&
         (int64_t)(2 + 2 * ns) * k * Q * kWave * 4 <= 65536)
    ns *= 2;
  return ns;
}

size_t nk_fwd_lds(int Q, int k, int ns) { return std::max<size_t>(16, ((size_t)k * Q + (size_t)ns * Q) * kWave * 4); }
size_t nk_bwd_lds(int Q, int k, int ns) { return std::max<size_t>(16, (size_t)(1 + ns) * k * Q * kWave * 4); }

// logits of every (parent, site); with `ce` on the small-grid path the
// cross-entropy runs in the same launch (returns true: no logits written)
bool launch_logits(const NkArgs& a, int ns, hipStream_t st, float* logits,
                   const NkCe* ce = nullptr) {
  if (nk_use_pp(a.R, a.L, a.Q, a.k, a.QK)) {
    const dim3 grid((unsigned)((int64_t)a.R * a.L));
    const NkCe c = ce ? *ce : NkCe{};
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(kNkPP), 0, st, a, logits, c); };
    if (ce) {
      if (a.Q == 2) go(nk_logits_pp_kernel<2, true>);
      else go(nk_logits_pp_kernel<4, true>);
    } else {
      if (a.Q == 2) go(nk_logits_pp_kernel<2, false>);
      else go(nk_logits_pp_kernel<4, false>);
    }
    return ce != nullptr;
  }
  if (nk_use_reg(a.Q, a.k)) {
    nk_reg_run(a, st, logits, nullptr, nullptr);
    return false;
  }
  const dim3 grid((a.R + kWave - 1) / kWave, a.L), block(kWave, ns);
  const size_t lds = nk_fwd_lds(a.Q, a.k, ns);
  switch (a.Q) {
    case 2: hipLaunchKernelGGL(nk_logits_kernel<2>, grid, block, lds, st, a, logits); break;
    case 4: hipLaunchKernelGGL(nk_logits_kernel<4>, grid, block, lds, st, a, logits); break;
    case 20: hipLaunchKernelGGL(nk_logits_kernel<20>, grid, block, lds, st, a, logits); break;
    default: hipLaunchKernelGGL(nk_logits_kernel<0>, grid, block, lds, st, a, logits);
  }
  return false;
}

void launch_logits_bwd(const NkArgs& a, int ns, hipStream_t st, const float* g, float* G) {
  if (nk_use_pp(a.R, a.L, a.Q, a.k, a.QK)) {
    const dim3 grid((unsigned)((int64_t)a.R * a.L));
    const size_t lds = (size_t)a.k * a.Q * kNkPP * 4;
    if (a.Q == 2)
      hipLaunchKernelGGL(nk_logits_bwd_pp_kernel<2>, grid, dim3(kNkPP), lds, st, a, g, G);
    else
      hipLaunchKernelGGL(nk_logits_bwd_pp_kernel<4>, grid, dim3(kNkPP), lds, st, a, g, G);
    return;
  }
  if (nk_use_reg(a.Q, a.k)) {
    nk_reg_run(a, st, nullptr, g, G);
    return;
  }
  const dim3 grid((a.R + kWave - 1) / kWave, a.L), block(kWave, ns);
  const size_t lds = nk_bwd_lds(a.Q, a.k, ns);
  switch (a.Q) {
    case 2: hipLaunchKernelGGL(nk_logits_bwd_kernel<2>, grid, block, lds, st, a, g, G); break;
    case 4: hipLaunchKernelGGL(nk_logits_bwd_kernel<4>, grid, block, lds, st, a, g, G); break;
    case 20: hipLaunchKernelGGL(nk_logits_bwd_kernel<20>, grid, block, lds, st, a, g, G); break;
    default: hipLaunchKernelGGL(nk_logits_bwd_kernel<0>, grid, block, lds, st, a, g, G);
  }
}

int grid1d(int64_t n, int block) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + block - 1) / block, 1 << 16)); }

// plan header ints
constexpr int kNkHeader = 16;

struct NkPlanView {
  int N, L, k, nP, n_nonroot;
  const int32_t *prow, *cofs, *cidx, *rowmap, *iofs, *ient;
};

NkPlanView plan_view(const int32_t* plan, int N, int L, int k, int nP) {
  NkPlanView v;
  v.N = N;
  v.L = L;
  v.k = k;
  v.nP = nP;
  v.n_nonroot = 0;
  const int32_t* p = plan + kNkHeader;
  v.prow = p;
  p += N;  // room for N distinct parents
  v.cofs = p;
  p += N + 1;
  v.cidx = p;
  p += N;
  v.rowmap = p;
  p += N;
  v.iofs = p;
  p += L + 1;
  v.ient = p;
  return v;
}

}  // namespace
}  // namespace trex

using namespace trex;

extern "C" int64_t trex_nk_plan_ints(int N, int L, int k) {
  if (N <= 0 || L <= 0 || k < 0) return 0;
  return kNkHeader + 4LL * N + 1 + (L + 1) + (int64_t)L * k;
}

extern "C" int trex_nk_plan_build(const int32_t* parent, int N, const int32_t* interactions,
                                  int L, int k, int32_t* plan, int32_t* info) {
  if (!parent || !plan || N <= 0 || L <= 0 || k < 0 || k > kNkMaxK || (k > 0 && !interactions))
    return set_error(TREX_E_ARG, "trex_nk_plan_build: bad arguments (N=%d L=%d k=%d)", N, L, k);
  for (int n = 0; n < N; ++n)
    if (parent[n] < 0 || parent[n] >= N)
      return set_error(TREX_E_ARG, "trex_nk_plan_build: parent[%d] = %d out of range", n, parent[n]);
  for (int64_t t = 0; t < (int64_t)L * k; ++t)
    if (interactions[t] < 0 || interactions[t] >= L)
      return set_error(TREX_E_ARG, "trex_nk_plan_build: interaction %lld = %d out of range",
                       (long long)t, interactions[t]);
  std::memset(plan, 0, sizeof(int32_t) * trex_nk_plan_ints(N, L, k));
  NkPlanView v = plan_view(plan, N, L, k, 0);
  int32_t* prow = const_cast<int32_t*>(v.prow);
  int32_t* cofs = const_cast<int32_t*>(v.cofs);
  int32_t* cidx = const_cast<int32_t*>(v.cidx);
  int32_t* rowmap = const_cast<int32_t*>(v.rowmap);
  int32_t* iofs = const_cast<int32_t*>(v.iofs);
  int32_t* ient = const_cast<int32_t*>(v.ient);
  // distinct parent rows (ascending) and their children (ascending)
  std::vector<int> cnt(N, 0);
  int nonroot = 0;
  for (int n = 0; n < N; ++n) {
    cnt[parent[n]] += 1;
    nonroot += parent[n] != n;
  }
  int nP = 0;
  for (int p = 0; p < N; ++p) {
    rowmap[p] = cnt[p] > 0 ? nP : -1;
    if (cnt[p] > 0) prow[nP++] = p;
  }
  cofs[0] = 0;
  for (int i = 0; i < nP; ++i) cofs[i + 1] = cofs[i] + cnt[prow[i]];
  std::vector<int> fill(nP, 0);
  for (int n = 0; n < N; ++n) {
    const int pc = rowmap[parent[n]];
    cidx[cofs[pc] + fill[pc]++] = n;
  }
  // inverse interactions: entries (site*k + j) grouped by the named site
  std::vector<int> icnt(L, 0);
  for (int64_t t = 0; t < (int64_t)L * k; ++t) icnt[interactions[t]] += 1;
  iofs[0] = 0;
  for (int m = 0; m < L; ++m) iofs[m + 1] = iofs[m] + icnt[m];
  std::vector<int> ifill(L, 0);
  for (int64_t t = 0; t < (int64_t)L * k; ++t) {
    const int m = interactions[t];
    ient[iofs[m] + ifill[m]++] = (int32_t)t;
  }
  plan[0] = kNkMagic;
  plan[1] = N;
  plan[2] = L;
  plan[3] = k;
  plan[4] = nP;
  plan[5] = nonroot;
  if (info) {
    info[0] = nP;
    info[1] = nonroot;
  }
  return TREX_OK;
}

extern "C" int64_t trex_nk_workspace_bytes(int N, int L, int Q, int k, int n_parents) {
  if (N <= 0 || L <= 0 || Q <= 0 || k < 0 || n_parents <= 0) return 0;
  const int64_t per = (int64_t)L * Q;
  int64_t b = 0;
  b += (int64_t)n_parents * per * 4;      // logits
  b += (int64_t)n_parents * per * 4;      // dlogits
  b += (int64_t)N * per * 4;              // dchild
  b += (int64_t)n_parents * per * k * 4;  // G
  b += (int64_t)n_parents * per * 4;      // dpar
  b += (int64_t)n_parents * L * 8;        // CE partials
  b += 256 * 8;                           // chunk sums
  return b + 7 * 256;
}

extern "C" int trex_nk_parental_logits(const float* seqs, const int32_t* rows, int R, int L, int Q,
                                       const int32_t* interactions, int k, const float* fitness,
                                       float* logits, void* stream) {
  const char* fn = "trex_nk_parental_logits";
  if (int e = nk_check(fn, L, Q, k)) return e;
  if (!seqs || !rows || R <= 0 || !fitness || !logits || (k > 0 && !interactions))
    return set_error(TREX_E_ARG, "%s: null pointer / bad R", fn);
  if (Q == 4 && (misaligned16(seqs) || misaligned16(logits)))
    return set_error(TREX_E_ARG, "%s: Q = 4 rows are read as float4: pointers must be 16-byte "
                     "aligned", fn);
  NkArgs a{seqs, rows, interactions, fitness, R, L, Q, k, (int)ipow(Q, k)};
  const int ns = nk_slices(R, L, Q, k);
  launch_logits(a, ns, (hipStream_t)stream, logits);
  return nk_err(fn);
}

extern "C" int trex_nk_landscape_loss(const int32_t* plan, int n_parents, const float* seqs, int N,
                                      int L, int Q, const int32_t* interactions, int k,
                                      const float* fitness, const float* seq_mask,
                                      float n_valid, float lambda_val, int n_nonroot,
                                      const float* surrogate, const float* d_seqs_in, float* loss,
                                      float* d_seqs, void* workspace, int64_t workspace_bytes,
                                      void* stream) {
  const char* fn = "trex_nk_landscape_loss";
  if (int e = nk_check(fn, L, Q, k)) return e;
  if (!plan || !seqs || !fitness || !loss || !workspace || n_parents <= 0 || N <= 0 ||
      (k > 0 && !interactions))
    return set_error(TREX_E_ARG, "%s: null pointer / bad sizes", fn);
  if (workspace_bytes < trex_nk_workspace_bytes(N, L, Q, k, n_parents))
    return set_error(TREX_E_ARG, "%s: workspace too small", fn);
  if (Q == 4 && (misaligned16(seqs) || misaligned16(d_seqs) || misaligned16(d_seqs_in) ||
                 misaligned16(workspace)))
    return set_error(TREX_E_ARG, "%s: Q = 4 rows are read as float4: pointers must be 16-byte "
                     "aligned", fn);
  if (!pos_finite_f32(n_valid) || n_nonroot <= 0)
    return set_error(TREX_E_ARG, "%s: empty normaliser (n_valid=%g, n_nonroot=%d)", fn, n_valid,
                     n_nonroot);
  hipStream_t st = (hipStream_t)stream;
  const NkPlanView v = plan_view(plan, N, L, k, n_parents);
  const int64_t per = (int64_t)L * Q;
  auto carve = [&](char*& p, int64_t bytes) {
    char* r = p;
    p += (bytes + 255) / 256 * 256;
    return r;
  };
  char* w = static_cast<char*>(workspace);
  float* logits = reinterpret_cast<float*>(carve(w, (int64_t)n_parents * per * 4));
  float* dlog = reinterpret_cast<float*>(carve(w, (int64_t)n_parents * per * 4));
  float* dchild = reinterpret_cast<float*>(carve(w, (int64_t)N * per * 4));
  float* G = reinterpret_cast<float*>(carve(w, (int64_t)n_parents * per * k * 4));
  float* dpar = reinterpret_cast<float*>(carve(w, (int64_t)n_parents * per * 4));
  double* part = reinterpret_cast<double*>(carve(w, (int64_t)n_parents * L * 8));
  double* sums = reinterpret_cast<double*>(carve(w, kNkChunks * 8));

  NkArgs a{seqs, v.prow, interactions, fitness, n_parents, L, Q, k, (int)ipow(Q, k)};
  const int ns = nk_slices(n_parents, L, Q, k);
  const double norm = (double)n_nonroot * (double)n_valid;
  const float scale = (float)((double)lambda_val / norm);
  const NkCe ce{seqs, v.cofs, v.cidx, seq_mask, scale, dlog, dchild, part};
  const char* v4e = std::getenv("TREX_NK_V4");  // "0": the generic kernels (A/B)
  const bool v4 = Q == 4 && !(v4e && v4e[0] == '0');
  if (!launch_logits(a, ns, st, logits, &ce)) {
    if (v4)
      hipLaunchKernelGGL(nk_ce4_kernel, dim3(grid1d((int64_t)n_parents * L, 256)), dim3(256), 0, st,
                         reinterpret_cast<const float4*>(seqs), reinterpret_cast<const float4*>(logits),
                         v.cofs, v.cidx, seq_mask, n_parents, L, scale,
                         reinterpret_cast<float4*>(dlog), reinterpret_cast<float4*>(dchild), part);
    else
      hipLaunchKernelGGL(nk_ce_kernel, dim3(grid1d((int64_t)n_parents * L, 256)), dim3(256), 0, st,
                         seqs, logits, v.cofs, v.cidx, seq_mask, n_parents, L, Q, scale, dlog,
                         dchild, part);
  }
  if (int e = nk_err(fn)) return e;
  // few (parent, site) partials (the eval shape: 465): one block sums them
  // directly; otherwise two fixed levels (chunks, then the chunk sums)
  const int64_t nparts = (int64_t)n_parents * L;
  if (nparts <= kNkDirectParts) {
    hipLaunchKernelGGL(nk_loss_kernel, dim3(1), dim3(256), 0, st, part, nparts, surrogate,
                       (double)lambda_val / norm, loss);
  } else {
    hipLaunchKernelGGL(nk_chunk_sum_kernel, dim3(kNkChunks), dim3(256), 0, st, part, nparts, sums);
    hipLaunchKernelGGL(nk_loss_kernel, dim3(1), dim3(256), 0, st, sums, (int64_t)kNkChunks,
                       surrogate, (double)lambda_val / norm, loss);
  }
  if (int e = nk_err(fn)) return e;
  if (!d_seqs) return TREX_OK;
  // the per-slot gradients G are gathered into each parent row inline by the
  // combine: for neighbour site m, the sum over the (site, j) entries naming
  // m (inverse CSR iofs / ient, ascending (site, j))
  if (k > 0) launch_logits_bwd(a, ns, st, dlog, G);
  (void)dpar;
  const int64_t glds = (int64_t)L * k * 16;
  // the LDS-staged combine wants up to kNkCombineLds of dynamic LDS: granted
  // once per process; a device (or an ARCH build) that refuses it runs the
  // plain combine instead
  static const int64_t lds_cap = [] {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(nk_combine4_lds_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kNkCombineLds) ==
        hipSuccess)
      return kNkCombineLds;
    (void)hipGetLastError();
    return (int64_t)65536;
  }();
  if (v4 && k > 0 && glds <= lds_cap) {
    hipLaunchKernelGGL(nk_combine4_lds_kernel, dim3(N), dim3(kNkCombineThreads), (size_t)glds, st,
                       reinterpret_cast<const float4*>(d_seqs_in),
                       reinterpret_cast<const float4*>(dchild), reinterpret_cast<const float4*>(G),
                       v.iofs, v.ient, v.rowmap, L, k, reinterpret_cast<float4*>(d_seqs));
  } else if (v4)
    hipLaunchKernelGGL(nk_combine4_kernel, dim3(grid1d((int64_t)N * L, 256)), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(d_seqs_in),
                       reinterpret_cast<const float4*>(dchild),
                       k > 0 ? reinterpret_cast<const float4*>(G) : nullptr, v.iofs, v.ient,
                       v.rowmap, N, L, k, reinterpret_cast<float4*>(d_seqs));
  else
    hipLaunchKernelGGL(nk_combine_kernel, dim3(grid1d((int64_t)N * per, 256)), dim3(256), 0, st,
                       d_seqs_in, dchild, k > 0 ? G : nullptr, v.iofs, v.ient, v.rowmap, N, L, Q,
                       k, d_seqs);
  return nk_err(fn);
}
