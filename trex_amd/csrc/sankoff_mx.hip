// libtrexhip.so -- matrix-core Sankoff kernel for 4 < Q <= 20 states (C3:
// protein, Q = 20), gfx950.
//
// Same semantics as sankoff_wide.hip (trex src/trex/sankoff.py run_dp
// :24-94, run_sankoff :114-188, the build-defined softmin adjoint), for the
// factored softmin (K = exp(-(C - cmin) / tau), range(C) / tau <= 40) with
// exact leaf messages -- the C3 configuration.  The other modes (hard, per-row
// stabilised softmin) stay on the state-parallel kernels: this kernel runs
// first, decides from the cost matrix on the device and publishes its
// decision in a workspace flag; the state-parallel launch behind it exits at
// once when the flag is set, the partial reduce picks this kernel's tiles.
//
// Mapping.  A work item is one tree x 16 sites, a workgroup of 8 waves that
// walks the tree's height-levelled program (plan.cpp stage_one_tree, the
// staged kernel's program): a stage's nodes go to different waves, the
// serial chain is the tree height.  Inside a wave, lane l holds site l % 16
// and quarter g = l / 16 of the states: states g P .. g P + P - 1 (P =
// ceil(Q / 4), 5 for Q = 20), P floats per vector -- every per-state
// operation is lane-local, cross-quarter reductions are two
// v_permlane32/16_swap steps (no LDS, no exchange buffers).
//
// The dense state x state products run on the matrix core, f32 in / f32
// accumulate (v_mfma_f32_16x16x4_f32: bit-for-bit a k-ordered fmaf chain,
// exact f32 products):
//   s = K u   (forward message and adjoint weights, sankoff.py:67-68)
//   t = K^T r (child cotangent)
// as D[16 x 16 sites] = A[16 states x 4] B[4 x 16 sites] per chunk: B is the
// data vector in the lane layout above (chunk c = state g P + c of lane
// quarter g), A a constant K slice per lane, and the output rows 4g .. 4g+3
// (+16: second block) land on the same lane quarter as the input states --
// no re-layout between consecutive products.
// dC accumulates per lane as P x Q running sums of r_i u_j (row i = the
// lane's states, column j = every state of its site, broadcast by the same
// permlane swaps), times K_ij once at the end (fp64).
//
// Every internal row keeps one LDS slot [P][64] floats: its D during the
// forward, its cotangent during the adjoint (written by its parent, which
// has read the D it needs from the HBM DP table -- the adjoint re-read the
// roofline counts); so a tree of n_int internal rows needs n_int * 64 * P * 4
// bytes (80 KB for C3's 63 rows at Q = 20).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "sankoff_dev.h"
#include "trex_common.h"
#include "wide_dev.h"

namespace trex {

namespace {

constexpr int kMW = kStageWaves;  // waves per workgroup
constexpr int kMS = 16;           // sites per work item (the MFMA's N)
constexpr int kMxMaxQ = 20;
constexpr int kXRow = 33;  // outer-product scratch row (32 states + 1 pad: conflict-free reads)

typedef float mf4 __attribute__((ext_vector_type(4)));

struct MArgs {
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
  int* flag;          // 1: this kernel handled the launch (workspace word)
};

// LDS floats of the row slots ([ni][P][64]; the dC partials [kMW][Q][Q]
// doubles reuse them at the end)
__host__ __device__ constexpr int mx_slot_floats(int ni, int P, int Q) {
  return ni * P * kWave > kMW * Q * Q * 2 ? ni * P * kWave : kMW * Q * Q * 2;
}

#ifdef TREX_MX_TIMING
// diagnostic build (tools/build_diag_mx.sh): wave 0 of each of the first
// 4096 workgroups stamps s_memtime at phase boundaries
__device__ unsigned long long g_mx_t[4096][24];
#define MX_STAMP(j)                                                      \
  do {                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 4096 && (j) < 24)               \
      g_mx_t[blockIdx.x][j] = __builtin_amdgcn_s_memtime();              \
  } while (0)
#else
#define MX_STAMP(j) \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ void mx_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- cross-quarter exchanges (the 4 lanes l % 16 of one site) ----
// o[q] = v of quarter q, in absolute quarter order on every lane:
// v_permlane32_swap pairs rows (0, 2) / (1, 3), v_permlane16_swap (0, 1) / (2, 3)
__device__ __forceinline__ void quarters(float v, float (&o)[4]) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(a[0], a[0], false, false);
  const auto c = __builtin_amdgcn_permlane16_swap(a[1], a[1], false, false);
  o[0] = __uint_as_float(b[0]);
  o[1] = __uint_as_float(b[1]);
  o[2] = __uint_as_float(c[0]);
  o[3] = __uint_as_float(c[1]);
}
// min / sum over the 4 quarters, the same bits on all 4 lanes
__device__ __forceinline__ float qmin(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float m = fminf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fminf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float qsum(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float m = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// first-index argmax over the quarters: (value, state) pairs, larger value,
// then lower state (the quarters hold increasing state ranges)
__device__ __forceinline__ void qargmax(float& v, int& i) {
  auto comb = [](float v0, int i0, float v1, int i1, float& vo, int& io) {
    const bool take1 = v1 > v0 || (v1 == v0 && i1 < i0);
    vo = take1 ? v1 : v0;
    io = take1 ? i1 : i0;
  };
  {
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const auto b = __builtin_amdgcn_permlane32_swap((unsigned)i, (unsigned)i, false, false);
    comb(__uint_as_float(a[0]), (int)b[0], __uint_as_float(a[1]), (int)b[1], v, i);
  }
  {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const auto b = __builtin_amdgcn_permlane16_swap((unsigned)i, (unsigned)i, false, false);
    comb(__uint_as_float(a[0]), (int)b[0], __uint_as_float(a[1]), (int)b[1], v, i);
  }
}

// first-index argmin over the quarters (smaller value, then lower state)
__device__ __forceinline__ void qargmin(float& v, int& i) {
  auto comb = [](float v0, int i0, float v1, int i1, float& vo, int& io) {
    const bool take1 = v1 < v0 || (v1 == v0 && i1 < i0);
    vo = take1 ? v1 : v0;
    io = take1 ? i1 : i0;
  };
  {
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const auto b = __builtin_amdgcn_permlane32_swap((unsigned)i, (unsigned)i, false, false);
    comb(__uint_as_float(a[0]), (int)b[0], __uint_as_float(a[1]), (int)b[1], v, i);
  }
  {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const auto b = __builtin_amdgcn_permlane16_swap((unsigned)i, (unsigned)i, false, false);
    comb(__uint_as_float(a[0]), (int)b[0], __uint_as_float(a[1]), (int)b[1], v, i);
  }
}

// y = M x on the matrix core: x in the lane layout (chunk c = the lane's
// state g P + c), A[b][c] this lane's slice of M (row block b), y back in
// the lane layout (y[4b + q] = row 4g + q of block b)
// (the A slices live in LDS, [(b P + c)][64 lanes]: 2 NB P registers fewer
// in a kernel whose dC accumulators already take P x 20)
template <int P>
__device__ __forceinline__ void mx_matvec(const float* kop, int lane, const float (&x)[P],
                                          float (&y)[P]) {
  constexpr int NB = (P + 3) / 4;
  float A[NB][P];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < P; ++c) A[b][c] = kop[(b * P + c) * kWave + lane];
  mf4 acc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] = mf4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int c = 0; c < P; ++c)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[b][c], x[c], acc[b], 0, 0, 0);
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * b + q < P) y[4 * b + q] = acc[b][q];
}

template <int P, int PHASE>
__device__ __forceinline__ void mx_body(const MArgs& A, float* lds) {
  constexpr int NB = (P + 3) / 4;
  constexpr bool FWD = (PHASE & 1) != 0;
  constexpr bool BWD = (PHASE & 2) != 0;
  const int Q = A.Q;
  const int ni = A.n_int;
  const int L = A.L;
  const int tree = blockIdx.x / A.tiles;
  const int tile = blockIdx.x - tree * A.tiles;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x % kWave;
  const int s16 = lane & 15;
  const int qg = lane >> 4;  // quarter
  const int site = tile * kMS + s16;
  const bool active = site < L;
  const float a = A.a, bcoef = A.bcoef;
  bool valid[P];  // this lane's state g P + t exists
#pragma unroll
  for (int t = 0; t < P; ++t) valid[t] = qg * P + t < Q;

  MX_STAMP(0);
  // ---- cost matrix into LDS (one load per thread), range on every wave
  // (the kernel's mode decision) ----
  float* cl = lds;  // [Q][Q], before anything else is laid out
  for (int e = threadIdx.x; e < Q * Q; e += kMW * kWave) cl[e] = A.cost[e];
  __syncthreads();
  float lmin = INFINITY, lmax = -INFINITY;
  for (int e = lane; e < Q * Q; e += kWave) {
    const float c = cl[e];
    lmin = fminf(lmin, c);
    lmax = fmaxf(lmax, c);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lmin = fminf(lmin, __shfl_xor(lmin, off, kWave));
    lmax = fmaxf(lmax, __shfl_xor(lmax, off, kWave));
  }
  const float cmin = uniform(lmin), cmax = uniform(lmax);
  const bool handled = use_ktrick(cmin, cmax, a) && (kSentinel - (cmax - cmin)) * a >= 64.0f;
  if (threadIdx.x == 0) __hip_atomic_store(A.flag, handled ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!handled) return;

  // ---- LDS: slots [ni][P][64] | K, K^T operand slices [2][NB P][64] |
  // tab [Q+1][Q] | ik [Q][Q] | sinv [Q] | leaf codes [nl][16] ----
  float* slots = lds;
  float* kop = slots + mx_slot_floats(ni, P, Q);
  float* ktop = kop + NB * P * kWave;
  float* tab = ktop + NB * P * kWave;
  float* ik = tab + (Q + 1) * Q;
  float* sinv = ik + Q * Q;
  float* kval = sinv + kMxMaxQ;  // K [Q][Q]
  float* cst = kval + kMxMaxQ * kMxMaxQ;  // the cost matrix, moved out of the slot area
  float* xscr = cst + kMxMaxQ * kMxMaxQ;  // per-wave outer-product scratch [kMW][2][16][kXRow]
  int8_t* lleaf = reinterpret_cast<int8_t*>(xscr + kMW * 2 * kMS * kXRow);
  for (int e = threadIdx.x; e < kMW * 2 * kMS * kXRow; e += kMW * kWave) xscr[e] = 0.0f;
  for (int e = threadIdx.x; e < Q * Q; e += kMW * kWave) cst[e] = cl[e];
  __syncthreads();
  auto slot = [&](int r, int t) -> float& { return slots[((size_t)r * P + t) * kWave + lane]; };

  // leaf message table (exact leaf weights: the message of a leaf observed
  // in state `code` is C[i][code]; row Q: the all-1e5 row's message), its
  // adjoint factors 1 / K[i][code], and 1 / sum_j K[i][j] (all-1e5 row)
  for (int e = threadIdx.x; e < Q * Q; e += kMW * kWave) {
    const int code = e / Q, i = e - code * Q;
    const float cv = cst[i * Q + code];
    tab[e] = cv;
    ik[e] = fast_exp2((cv - cmin) * a);
    kval[e] = fast_exp2((cmin - cst[e]) * a);
  }
  if (threadIdx.x < Q) {
    const int i = threadIdx.x;
    float sk = 0.0f;
    for (int j = 0; j < Q; ++j) sk += fast_exp2((cmin - cst[i * Q + j]) * a);
    tab[Q * Q + i] = fmaf(-bcoef, fast_log2(sk), kSentinel + cmin);
    sinv[i] = __builtin_amdgcn_rcpf(sk);
  }
  {
    const int8_t* lv = A.leaves + (size_t)tree * A.nl * L;
    for (int e = threadIdx.x; e < A.nl * kMS; e += kMW * kWave) {
      const int leaf = e / kMS;
      const int s = tile * kMS + (e - leaf * kMS);
      int code = s < L ? (int)lv[(size_t)leaf * L + s] : Q;
      code = ((unsigned)code < (unsigned)Q) ? code : Q;
      lleaf[e] = (int8_t)code;
    }
  }
  // every lane's slices of K and K^T (rows: output block b, lane row
  // l % 16 -> state (l % 16 / 4) P + 4 b + l % 4; columns: chunk c,
  // k = l / 16 -> state k P + c)
  for (int e = threadIdx.x; e < 2 * NB * P * kWave; e += kMW * kWave) {
    const int l = e % kWave, bc = (e / kWave) % (NB * P), tr = e / (NB * P * kWave);
    const int b = bc / P, c = bc - b * P;
    const int to = 4 * b + (l & 3);
    const int so = ((l & 15) >> 2) * P + to;
    const int si = (l >> 4) * P + c;
    const bool ok = to < P && so < Q && si < Q;
    kop[e] = ok ? fast_exp2((cmin - cst[tr ? si * Q + so : so * Q + si]) * a) : 0.0f;
  }
  __syncthreads();

  MX_STAMP(1);
  // program: steps of stage s on wave w are [off[s W + w], off[s W + w + 1])
  const cptr<int> prog = as_const(A.staged) + (size_t)tree * A.stride;
  const int S = prog[4 * ni];
  const cptr<int> offs = prog + 4 * ni + 1;
  // this wave's step words in its lanes (lane t = its t-th step, stages in
  // order) when they fit in 64, read with v_readlane: no scalar load on the
  // step chain (sankoff_staged.hip does the same)
  int vlo = 0, vhi = 0, vsb = 0, sx = 0, sy = 0, sz = 0, sw = 0;
  bool regsteps;
  {
    if (lane < S) {
      vlo = offs[lane * kMW + wv];
      vhi = offs[lane * kMW + wv + 1];
    }
    const int cnt = vhi - vlo;
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int t = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += t;
    }
    vsb = incl - cnt;
    const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
    regsteps = S <= kWave && total <= kWave;
    if (regsteps) {
      int k = -1;
      for (int s2 = 0; s2 < S; ++s2) {
        const int b = __builtin_amdgcn_readlane(vsb, s2);
        const int lo2 = __builtin_amdgcn_readlane(vlo, s2);
        const int c2 = __builtin_amdgcn_readlane(vhi, s2) - lo2;
        if (lane >= b && lane < b + c2) k = lo2 + lane - b;
      }
      if (k >= 0) {
        const int* e = A.staged + (size_t)tree * A.stride + 4 * k;
        sx = e[0];
        sy = e[1];
        sz = e[2];
        sw = e[3];
      }
    }
  }
  // step k of stage s (lo = the stage's first step on this wave)
  auto get_step = [&](int s, int lo, int k) -> I4 {
    if (regsteps) {
      const int t = __builtin_amdgcn_readlane(vsb, s) + k - lo;
      return I4{__builtin_amdgcn_readlane(sx, t), __builtin_amdgcn_readlane(sy, t),
                __builtin_amdgcn_readlane(sz, t), __builtin_amdgcn_readlane(sw, t)};
    }
    return load_step(prog, k);
  };
  auto stage_lo = [&](int s) { return regsteps ? __builtin_amdgcn_readlane(vlo, s) : offs[s * kMW + wv]; };
  auto stage_hi = [&](int s) { return regsteps ? __builtin_amdgcn_readlane(vhi, s) : offs[s * kMW + wv + 1]; };

  const uint32_t rowbytes = (uint32_t)L * Q * 4;
  const uint32_t treebytes = (uint32_t)ni * rowbytes;
  const rsrc_t rdp = make_rsrc(A.dp + (size_t)tree * ni * L * Q, treebytes);
  // byte offset of (site, state g P + t) in a row; past the buffer when absent
  const int vbase = active ? (site * Q + qg * P) * 4 : 0x7FFFFFF0;
  auto voff = [&](int t) { return valid[t] ? vbase + 4 * t : 0x7FFFFFF0; };

  // message of an internal child with D = d (lane layout) to every parent state
  // softmin weights of a child with D = d: md = min_j D_j (the stabiliser),
  // u_j = exp2((md - D_j) a), s_i = sum_j K_ij u_j.  The first-index argmin
  // j* has u = 1 exactly and is the dominant term: it is left out of the
  // matrix-core chain and added last (s_i = K_ij* + sum_{j != j*} K_ij u_j),
  // so the small terms sum among themselves instead of being absorbed one by
  // one into ~1 (each such absorption rounds the same way: a bias of ~1e-7
  // per message, 2e-6 per C3 site score after 62 messages -- measured)
  auto weights = [&](const float (&d)[P], float& md, float (&u)[P], float (&sv)[P]) {
    float lm = INFINITY;
    int li = 0;
#pragma unroll
    for (int t = 0; t < P; ++t)
      if (valid[t] && d[t] < lm) {
        lm = d[t];
        li = qg * P + t;
      }
    qargmin(lm, li);
    md = lm;
    float ux[P];
#pragma unroll
    for (int t = 0; t < P; ++t) {
      u[t] = valid[t] ? fast_exp2((md - d[t]) * a) : 0.0f;
      ux[t] = qg * P + t == li ? 0.0f : u[t];
    }
    mx_matvec<P>(kop, lane, ux, sv);
#pragma unroll
    for (int t = 0; t < P; ++t) sv[t] += valid[t] ? kval[(qg * P + t) * Q + li] : 0.0f;
  };
  auto message = [&](const float (&d)[P], float (&m)[P]) {
    float md, u[P], sv[P];
    weights(d, md, u, sv);
#pragma unroll
    for (int t = 0; t < P; ++t) m[t] = valid[t] ? fmaf(-bcoef, fast_log2(sv[t]), md + cmin) : 0.0f;
  };
  auto leaf_message = [&](int code, float (&m)[P]) {
#pragma unroll
    for (int t = 0; t < P; ++t) m[t] = valid[t] ? tab[code * Q + qg * P + t] : 0.0f;
  };

  // ---- forward: stage by stage, each wave its own node list ----
  if constexpr (FWD) {
    for (int s = 0; s < S; ++s) {
      const int lo = stage_lo(s), hi = stage_hi(s);
      for (int k = lo; k < hi; ++k) {
        const I4 stp = get_step(s, lo, k);
        float dv[P];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? stp.y : stp.z;
          const int kind = (desc >> 24) & 3;
          float m[P];
          if (kind == kKindLeaf) {
            leaf_message(lleaf[(desc & 0xFFFF) * kMS + s16], m);
          } else if (kind == kKindInt) {
            float d[P];
#pragma unroll
            for (int t = 0; t < P; ++t) d[t] = slot(desc & 0xFFFF, t);
            message(d, m);
          } else {
            leaf_message(Q, m);
          }
#pragma unroll
          for (int t = 0; t < P; ++t) dv[t] = (c == 0) ? m[t] : dv[t] + m[t];
        }
        const int row = stp.x & 0xFFFF;
#pragma unroll
        for (int t = 0; t < P; ++t) {
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dv[t]), rdp, voff(t), row * rowbytes, 0);
          slot(row, t) = dv[t];
        }
      }
      mx_lds_barrier();
      MX_STAMP(2 + (s < 6 ? s : 5));
    }
  }

  // ---- root (last internal row): score + cotangent (sankoff.py:187), wave 0 ----
  if (wv == 0) {
    float dv[P];
    if constexpr (FWD) {
#pragma unroll
      for (int t = 0; t < P; ++t) dv[t] = slot(ni - 1, t);
    } else {
#pragma unroll
      for (int t = 0; t < P; ++t)
        dv[t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rdp, voff(t), (ni - 1) * rowbytes, 1));
    }
    float lm = INFINITY;
#pragma unroll
    for (int t = 0; t < P; ++t) lm = valid[t] ? fminf(lm, dv[t]) : lm;
    const float mn = qmin(lm);
    float gr[P], score;
    if (A.hard_root) {
      float lc = 0.0f;
#pragma unroll
      for (int t = 0; t < P; ++t) lc += (valid[t] && dv[t] == mn) ? 1.0f : 0.0f;
      const float cnt = qsum(lc);
#pragma unroll
      for (int t = 0; t < P; ++t) gr[t] = (valid[t] && dv[t] == mn) ? 1.0f / cnt : 0.0f;
      score = mn;
    } else {
      // sum of exp2((mn - D) a): the minima (exactly 1 each) are counted
      // apart and added last, the small terms sum among themselves first
      float e[P], ls = 0.0f, lt = 0.0f;
#pragma unroll
      for (int t = 0; t < P; ++t) {
        e[t] = valid[t] ? fast_exp2((mn - dv[t]) * a) : 0.0f;
        const bool tie = valid[t] && dv[t] == mn;
        ls += tie ? 0.0f : e[t];
        lt += tie ? 1.0f : 0.0f;
      }
      const float sum = qsum(lt) + qsum(ls);
      const float rs = __builtin_amdgcn_rcpf(sum);
#pragma unroll
      for (int t = 0; t < P; ++t) gr[t] = e[t] * rs;
      score = fmaf(-bcoef, fast_log2(sum), mn);
    }
    if constexpr (FWD) {
      const bool leader = active && qg == 0;
      if (leader && A.site_score) A.site_score[(size_t)tree * L + site] = score;
      const double tot = wave_sum(leader ? (double)score : 0.0);
      if (lane == 0) A.part_tree[blockIdx.x] = tot;
    }
    if constexpr (BWD) {
      const float dscale = A.dts ? as_const(A.dts)[tree] : 1.0f;
#pragma unroll
      for (int t = 0; t < P; ++t) slot(ni - 1, t) = active ? gr[t] * dscale : 0.0f;
    }
  }

  if constexpr (BWD) {
    // the forward's DP stores of every wave must be in L2 before any wave
    // re-reads them (loads below bypass L1: glc)
    if constexpr (FWD) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    MX_STAMP(8);
    // dC accumulates on the matrix core: per child, the wave's (r, u) pairs
    // go through its LDS scratch [16 sites][33] (r | u), read back as
    // 16x16x4 f32 operands (k = 4 sites) -- acc_ij += sum_sites r_i u_j,
    // 2 x 2 blocks of 16 x 16 (i, j < 32), x K_ij at the end (fp64)
    mf4 oacc[2][2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) oacc[ib][jb] = mf4{0.0f, 0.0f, 0.0f, 0.0f};
    float* xr = xscr + (size_t)wv * 2 * kMS * kXRow;
    float* xu = xr + kMS * kXRow;
    auto outer = [&](const float (&r)[P], const float (&u)[P]) {
#pragma unroll
      for (int t = 0; t < P; ++t)
        if (valid[t]) {
          xr[s16 * kXRow + qg * P + t] = r[t];
          xu[s16 * kXRow + qg * P + t] = u[t];
        }
      wave_sync();
#pragma unroll
      for (int kc = 0; kc < kMS / 4; ++kc) {
        const int pr = (4 * kc + (lane >> 4)) * kXRow + (lane & 15);
        float ra[2], ub[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ra[h] = xr[pr + 16 * h];
          ub[h] = xu[pr + 16 * h];
        }
#pragma unroll
        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
          for (int jb = 0; jb < 2; ++jb)
            oacc[ib][jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[ib], ub[jb], oacc[ib][jb], 0, 0, 0);
      }
      wave_sync();
    };
    const bool want_marg = A.marg != nullptr;
    const rsrc_t rmg = make_rsrc(want_marg ? A.marg + (size_t)tree * ni * L * Q : A.dp, treebytes);
    int8_t* at = A.anc ? A.anc + (size_t)tree * ni * L + site : nullptr;

    // the wave's adjoint steps in order (stages S-1 .. 0, each hi-1 .. lo):
    // the children's DP rows of the NEXT step are loaded while this one
    // computes (HBM / L2, glc; the table is final, so across stage barriers
    // too); non-internal children load nothing (offset past the buffer)
    // (s, k) of the step after (s, k) in this order, or k = -1
    auto next_step = [&](int s, int k, int& s_out) {
      s_out = s;
      if (k > stage_lo(s)) return k - 1;
      for (int s2 = s - 1; s2 >= 0; --s2)
        if (stage_hi(s2) > stage_lo(s2)) {
          s_out = s2;
          return stage_hi(s2) - 1;
        }
      return -1;
    };
    auto load_children = [&](int s2, int k, float (&dc)[2][P]) {
      const I4 st2 = k >= 0 ? get_step(s2, stage_lo(s2), k) : I4{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int desc = c == 0 ? st2.y : st2.z;
        const bool internal = k >= 0 && ((desc >> 24) & 3) == kKindInt;
        const int crow = internal ? (desc & 0xFFFF) : 0;
#pragma unroll
        for (int t = 0; t < P; ++t)
          dc[c][t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              rdp, internal ? voff(t) : 0x7FFFFFF0, crow * rowbytes, 1));
      }
    };
    float ndc[2][P];
    {
      int k0 = -1, s0 = 0;
      for (int s2 = S - 1; s2 >= 0 && k0 < 0; --s2)
        if (stage_hi(s2) > stage_lo(s2)) {
          k0 = stage_hi(s2) - 1;
          s0 = s2;
        }
      load_children(s0, k0, ndc);
    }
    for (int s = S - 1; s >= 0; --s) {
      const int lo = stage_lo(s), hi = stage_hi(s);
      for (int k = hi - 1; k >= lo; --k) {
        const I4 stp = get_step(s, lo, k);
        float dc[2][P];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int t = 0; t < P; ++t) dc[c][t] = ndc[c][t];
        int sn;
        const int kn = next_step(s, k, sn);
        load_children(sn, kn, ndc);
        if (stp.w & kStepUnreached) continue;
        const int row = stp.x & 0xFFFF;
        float g[P];
#pragma unroll
        for (int t = 0; t < P; ++t) g[t] = slot(row, t);
        if (want_marg) {
#pragma unroll
          for (int t = 0; t < P; ++t)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g[t]), rmg, voff(t), row * rowbytes, 0);
        }
        if (at) {
          float bv = -INFINITY;
          int bi = 0;
#pragma unroll
          for (int t = 0; t < P; ++t)
            if (valid[t] && g[t] > bv) {
              bv = g[t];
              bi = qg * P + t;
            }
          qargmax(bv, bi);
          if (active && qg == 0) at[(size_t)row * L] = (int8_t)bi;
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? stp.y : stp.z;
          const int kind = (desc >> 24) & 3;
          if (kind == kKindInt) {
            // w_ij = K_ij u_j / s_i: r_i = g_i / s_i, acc_ij += r_i u_j,
            // child cotangent gc_j = u_j sum_i K_ij r_i
            float md, u[P], sv[P], r[P], tv[P];
            weights(dc[c], md, u, sv);
#pragma unroll
            for (int t = 0; t < P; ++t) r[t] = valid[t] ? g[t] * __builtin_amdgcn_rcpf(sv[t]) : 0.0f;
            mx_matvec<P>(ktop, lane, r, tv);
            outer(r, u);
            const int crow = desc & 0xFFFF;
#pragma unroll
            for (int t = 0; t < P; ++t) {
              float gc = u[t] * tv[t];
              if (desc & kStepAccumulate) gc += slot(crow, t);
              slot(crow, t) = gc;
            }
          } else {
            const int code = kind == kKindLeaf ? (int)lleaf[(desc & 0xFFFF) * kMS + s16] : Q;
            // present state: one-hot weight w_ij = [j == code]: acc_i,code +=
            // g_i / K_i,code; missing state / sentinel row (all 1e5): w_ij =
            // K_ij / sum_j K_ij, acc_ij += g_i / sum_j K_ij for every j
            float r[P], u[P];
#pragma unroll
            for (int t = 0; t < P; ++t) {
              const int st = qg * P + t;
              r[t] = !valid[t] ? 0.0f : code < Q ? g[t] * ik[code * Q + st] : g[t] * sinv[st];
              u[t] = (code == Q || st == code) ? 1.0f : 0.0f;
            }
            outer(r, u);
          }
        }
      }
      mx_lds_barrier();
      MX_STAMP(9 + (S - 1 - s < 6 ? S - 1 - s : 5));
    }

    // ---- dC partial of the item: each wave's blocks (already summed over
    // the 16 sites by the MFMAs), then the waves in order through LDS (the
    // slots are dead now) ----
    double* red = reinterpret_cast<double*>(slots);  // [kMW][Q][Q]
    const int Q2 = Q * Q;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = ib * 16 + 4 * (lane >> 4) + q, j = jb * 16 + (lane & 15);
          if (i < Q && j < Q) red[(size_t)wv * Q2 + i * Q + j] = (double)oacc[ib][jb][q];
        }
    __syncthreads();
    const int nb = A.B * A.tiles;
    for (int e = threadIdx.x; e < Q2; e += kMW * kWave) {
      double tsum = red[e];
#pragma unroll
      for (int w = 1; w < kMW; ++w) tsum += red[(size_t)w * Q2 + e];
      const int i = e / Q, j = e - i * Q;
      A.part_dc[(size_t)e * nb + blockIdx.x] = tsum * (double)fast_exp2((cmin - cst[i * Q + j]) * a);
    }
    MX_STAMP(15);
  }
}

template <int P, int PHASE>
__global__ __launch_bounds__(kMW * kWave, 1) void sankoff_mx_kernel(MArgs A) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  mx_body<P, PHASE>(A, lds);
}

template <int P>
void launch_mx_p(int phase, int grid, size_t lds, hipStream_t st, const MArgs& A) {
  auto go = [&](auto kernel) {
    if (lds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kMW * kWave), lds, st, A);
  };
  if (phase == 1)
    go(sankoff_mx_kernel<P, 1>);
  else if (phase == 2)
    go(sankoff_mx_kernel<P, 2>);
  else
    go(sankoff_mx_kernel<P, 3>);
}

}  // namespace

#ifdef TREX_MX_TIMING
extern "C" int trex_debug_mx_times(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mx_t), sizeof(g_mx_t)) == hipSuccess ? 0 : -4;
}
#endif

int mx_tiles(int L) { return (L + kMS - 1) / kMS; }

size_t mx_lds_bytes(int ni, int nl, int Q) {
  const int P = (Q + 3) / 4, NB = (P + 3) / 4;
  const size_t b = ((size_t)mx_slot_floats(ni, P, Q) + 2 * NB * P * kWave + (Q + 1) * Q + Q * Q +
                    kMxMaxQ + 2 * kMxMaxQ * kMxMaxQ + kMW * 2 * kMS * kXRow) * 4 +
                   (size_t)nl * kMS;
  return (b + 15) & ~(size_t)15;
}

// host-side eligibility (everything the host knows; the cost-dependent mode
// is decided in the kernel): soft, 4 < Q <= 20, the slots fit.  Opt-in
// (TREX_MX=1) until it beats the state-parallel kernel: measured on C3
// (tools/mx_check.py, tools/mx_times.py) 200 us against 150 us (229 us with
// the earlier VALU outer product, which spilled) -- 148k cycles per
// workgroup, one workgroup per CU (the D slots alone take 80 KB of LDS), 625
// tiles = 3 rounds on 256 CUs; the staged node chain is latency-bound at 2
// waves per SIMD; DESIGN.md section 5.8.
bool mx_eligible(const WideCall& c) {
  if (!c.soft || c.Q <= 4 || c.Q > kMxMaxQ) return false;
  const char* e = std::getenv("TREX_MX");  // read per call (tests flip it)
  if (!(e && e[0] == '1')) return false;
  if ((int64_t)c.ni * c.L * c.Q * 4 > 0x7FFFFFF0LL) return false;
  return mx_lds_bytes(c.ni, c.nl, c.Q) <= 160 * 1024;
}

int mx_run(const char* fn, const WideCall& c, const int32_t* staged, int* flag) {
  const int tiles = mx_tiles(c.L);
  const size_t lds = mx_lds_bytes(c.ni, c.nl, c.Q);
  if ((int64_t)c.B * tiles > 0x7FFFFFFF) return set_error(TREX_E_ARG, "%s: grid too large", fn);
  MArgs A;
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
  A.flag = flag;
  hipStream_t st = (hipStream_t)c.stream;
  const int grid = (int)nb;
  switch ((c.Q + 3) / 4) {
    case 2: launch_mx_p<2>(c.phase, grid, lds, st, A); break;
    case 3: launch_mx_p<3>(c.phase, grid, lds, st, A); break;
    case 4: launch_mx_p<4>(c.phase, grid, lds, st, A); break;
    default: launch_mx_p<5>(c.phase, grid, lds, st, A); break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

}  // namespace trex
