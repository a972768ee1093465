// libtrexhip.so -- the lane-per-site Sankoff kernel with each site's states
// split over a PAIR of waves, 4 < Q <= 20 (C3: protein, Q = 20), gfx950.
//
// Same semantics, task program, tables and results as sankoff_site.hip (trex
// src/trex/sankoff.py run_dp :24-94, run_sankoff :114-188, the build-defined
// softmin adjoint; DP table, scores, marginals and ancestral states bitwise
// that kernel's, dC within rtol 1e-5 of the fp64 oracle).  What changes is
// the mapping: a workgroup of 16 waves is 8 wave PAIRS, and the two waves of
// a pair (2p, 2p + 1) hold states 0..9 and 10..19 of the same 64 sites.
//
// Why not two lanes of one wave: the mat-vecs s = K u and t = K^T r take
// their K entries from SGPRs (one value per wave-instruction), and lanes
// holding different states would need different K entries in the same
// instruction.  Two waves can: wave h reads K rows 10h .. 10h + 9.  Per
// mat-vec each wave publishes its 10 u (or r) values in the pair's LDS
// scratch, the pair meets at an LDS flag (pair_sync), and each wave sums
// over all 20 j in the original order -- bitwise the same s_i / t_j.  Half
// the registers per lane (<= 128 VGPRs: 4 waves per SIMD), half the per-wave
// exp / log / rcp / FMA chain; the pair's syncs are the price.
//
// dC: each wave runs the outer-product / leaf-histogram MFMAs of half of
// the 64 sites (k-steps 2h, 2h + 1) into its own accumulators; the 16 waves'
// partials sum in a fixed order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "sankoff_dev.h"
#include "trex_common.h"
#include "wide_dev.h"

namespace trex {

namespace {

constexpr int kSQ2 = kSiteSQ;                 // states of a site (Q padded to 20)
constexpr int kH = kSQ2 / 2;                  // states per wave
constexpr int kSlotF2 = kSQ2 * kWave;         // floats per slot / scratch vector
constexpr int kTabF2 = (kSQ2 + 1) * kSQ2 + kSQ2;  // T[Q + 1][kSQ] + 1 / sum_j K_ij
constexpr int kScrF = kSQ2 * (kWave + 4) - 4;  // floats per pair scratch vector (padded rows; the last row's pad dropped)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

// eight floats (two float4 at p0, p1) split exactly into truncated bf16
// pieces x = h + m + l, packed two per dword in k order (sankoff_site.hip)
__device__ __forceinline__ void split3p(const float* p0, const float* p1, u32x4& h, u32x4& m,
                                        u32x4& l) {
  const float4 a = *reinterpret_cast<const float4*>(p0), b = *reinterpret_cast<const float4*>(p1);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const f2 x = pk(v[2 * q], v[2 * q + 1]);
    const u2 xb = __builtin_bit_cast(u2, x);
    const f2 r1 = x - __builtin_bit_cast(f2, xb & 0xFFFF0000u);
    const u2 mb = __builtin_bit_cast(u2, r1) & 0xFFFF0000u;
    const u2 lb = __builtin_bit_cast(u2, r1 - __builtin_bit_cast(f2, mb));
    h[q] = __builtin_amdgcn_perm(xb.y, xb.x, 0x07060302u);
    m[q] = __builtin_amdgcn_perm(mb.y, mb.x, 0x07060302u);
    l[q] = __builtin_amdgcn_perm(lb.y, lb.x, 0x07060302u);
  }
}


struct Site2Args {
  const int* lanes;
  int64_t stride;
  const int8_t* leaves;
  const float* cost;
  int n_int, nl, L, tiles, B, Q;
  float a, bcoef;
  int hard_root;
  float* dp;
  float* site_score;
  const float* dts;
  float* marg;
  int8_t* anc;
  double* part_tree;
  double* part_dc;
  const float* kg;
  const float* ptab;
  float* srow;
  const int* flag;
  int n_slots;
};

#ifdef TREX_SITE2_TIMING
// diagnostic build (tools/build_ab.sh s2t sankoff_site2.hip -DTREX_SITE2_TIMING):
// lane 0 of every wave of the first 2048 workgroups stamps s_memtime at the
// phase boundaries of sankoff_site.hip's SITE_STAMP (tools/site_times.py --pair)
__device__ unsigned long long g_site2_t[2048][16][20];
#define SITE2_STAMP(j)                                                             \
  do {                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 2048 && (j) < 20)                  \
      g_site2_t[blockIdx.x][threadIdx.x >> 6][j] = __builtin_amdgcn_s_memtime();  \
  } while (0)
#else
#define SITE2_STAMP(j) \
  do {                 \
  } while (0)
#endif

__device__ __forceinline__ void site2_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// transposed scratch rows padded to 68 floats: row i, site s at i * 68 + s.
// 16 rows read at one site group start in 16 distinct 16-byte bank groups
// (the XOR swizzle of sankoff_site.hip, but affine: every row's address is
// one base register plus an immediate offset -- no per-row address VGPRs)
constexpr int kRS = kWave + 4;
__device__ __forceinline__ int swz2(int i, int s) { return i * kRS + s; }

// NP: wave pairs per workgroup (8: 4 waves / SIMD at <= 128 VGPRs; 6: 3 at
// <= 168; 4: 2 -- the largest whose LDS fits, site2_run)
template <int PHASE, int QC, bool KS, int NP>
__global__ __launch_bounds__(2 * NP * kWave, 1) void sankoff_site2_kernel(Site2Args A) {
  constexpr int kPairs = NP;
  constexpr int kSW2 = 2 * NP;                  // waves per workgroup
  constexpr int kExF = 2 * NP * 2 * kWave;      // exchange: [2 bufs][pair][half][64]
  constexpr bool FWD = (PHASE & 1) != 0;
  constexpr bool BWD = (PHASE & 2) != 0;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (!__builtin_amdgcn_readfirstlane(as_const(A.flag)[0])) return;
  SITE2_STAMP(0);
  const int Q = QC ? QC : A.Q;
  const int ni = A.n_int;
  const int L = A.L;
  const int tree = blockIdx.x / A.tiles;
  const int tile = blockIdx.x - tree * A.tiles;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int pr = wv >> 1, hf = wv & 1;  // pair, half (states 10 hf .. 10 hf + 9)
  const int s0 = kH * hf;
  const int lane = threadIdx.x % kWave;
  const int site = tile * kWave + lane;
  const bool active = site < L;
  const float a = A.a, bcoef = A.bcoef;
  const cptr<float> K = as_const(A.kg);
  auto valid = [&](int k) { return s0 + k < Q; };

  // ---- LDS: slots [n_slots][kSQ][64] | pair scratch [8][2][kSQ][64] |
  // exchange [2][8][2][64] | flags [16] (+pad) | T, sinv | program | leaf codes ----
  float* slots = lds;
  float* scr = slots + (size_t)A.n_slots * kSlotF2;
  float* xr = scr + (size_t)pr * 2 * kScrF;
  float* xu = xr + kScrF;
  float* ex = scr + (size_t)kPairs * 2 * kScrF;
  volatile int* flags = reinterpret_cast<volatile int*>(ex + kExF);  // [16]
  float* tab = ex + kExF + 16;
  float* sinv = tab + (kSQ2 + 1) * kSQ2;
  int* lprog = reinterpret_cast<int*>(tab + kTabF2);
  const int pints = (int)A.stride;
  int8_t* lleaf = reinterpret_cast<int8_t*>(lprog + pints);

  // ---- the pair's meeting point: each wave's LDS writes done, its counter
  // published, the partner's counter waited for (counters only grow; a spin
  // that runs out flags the launch instead of hanging the GPU) ----
  int sync_n = 0;
  auto pair_sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ++sync_n;
    flags[wv] = sync_n;
#ifndef SITE2_DIAG_NOSYNC  // diagnostic: no waiting for the partner (wrong results; the syncs' cost)
    int guard = 0;
    while (__builtin_amdgcn_readfirstlane(flags[wv ^ 1]) < sync_n) {
#ifndef SITE2_NOSLEEP
      __builtin_amdgcn_s_sleep(1);
#endif
      if (++guard > (1 << 22)) break;  // never expected: the results are then wrong (tests)
    }
#endif
    asm volatile("" ::: "memory");
  };
  // one value per lane to the partner (two alternating buffers: a buffer is
  // rewritten only two exchanges later, after a sync the partner has passed
  // past its read)
  int ex_par = 0;
  auto exchange = [&](float v) -> float {
    float* e = ex + ((size_t)ex_par * kPairs + pr) * 2 * kWave;
    e[hf * kWave + lane] = v;
    pair_sync();
    const float o = e[(hf ^ 1) * kWave + lane];
    ex_par ^= 1;
    return o;
  };

  float cmin;
  {
    float lmin = INFINITY;
    for (int e = lane; e < Q * Q; e += kWave) lmin = fminf(lmin, A.cost[e]);
    cmin = uniform(wave_minf(lmin));
  }
  for (int e = threadIdx.x; e < (kSQ2 + 1) * kSQ2; e += kSW2 * kWave) {
    const int code = e / kSQ2, i = e - code * kSQ2;
    float v = 0.0f;
    if (i < Q) {
      if (code < Q) {
        v = A.cost[i * Q + code];
      } else {
        float sk = 0.0f;
        for (int j = 0; j < Q; ++j) sk += A.kg[i * kSQ2 + j];
        v = fmaf(-bcoef, fast_log2(sk), kSentinel + cmin);
      }
    }
    tab[e] = v;
  }
  if (threadIdx.x < kSQ2) {
    const int i = threadIdx.x;
    float sk = 0.0f;
    for (int j = 0; j < Q; ++j) sk += A.kg[i * kSQ2 + j];
    sinv[i] = i < Q ? __builtin_amdgcn_rcpf(sk) : 0.0f;
  }
  if (threadIdx.x < kSW2) flags[threadIdx.x] = 0;
  {
    const int* pg = A.lanes + (size_t)tree * A.stride;
    for (int e = threadIdx.x; e < pints; e += kSW2 * kWave) lprog[e] = pg[e];
    const int8_t* lv = A.leaves + (size_t)tree * A.nl * L;
    auto norm = [&](int code) { return ((unsigned)code < (unsigned)Q) ? code : Q; };
    if ((L & 3) == 0) {
      for (int e = threadIdx.x; e < A.nl * (kWave / 4); e += kSW2 * kWave) {
        const int leaf = e / (kWave / 4);
        const int c0 = tile * kWave + 4 * (e - leaf * (kWave / 4));
        uint32_t w = 0xFFFFFFFFu;
        if (c0 < L) w = *reinterpret_cast<const uint32_t*>(lv + (size_t)leaf * L + c0);
        uint32_t o = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) o |= (uint32_t)norm((int)(int8_t)(w >> (8 * q))) << (8 * q);
        reinterpret_cast<uint32_t*>(lleaf)[e] = o;
      }
    } else {
      for (int e = threadIdx.x; e < A.nl * kWave; e += kSW2 * kWave) {
        const int leaf = e / kWave;
        const int s = tile * kWave + (e - leaf * kWave);
        lleaf[e] = (int8_t)(s < L ? norm((int)lv[(size_t)leaf * L + s]) : Q);
      }
    }
  }
  __syncthreads();
  SITE2_STAMP(1);

  auto pword = [&](int e) { return __builtin_amdgcn_readfirstlane(lprog[e]); };
  const int S = pword(0);
  const int steps = 8 + ((ni + 1 + 3) & ~3);  // lp_steps_offset(ni)
  const int inl = steps + 4 * pword(2);
  auto load_step = [&](int base, int k) -> I4 {
    const int4 w = *reinterpret_cast<const int4*>(lprog + base + 4 * k);
    return I4{__builtin_amdgcn_readfirstlane(w.x), __builtin_amdgcn_readfirstlane(w.y),
              __builtin_amdgcn_readfirstlane(w.z), __builtin_amdgcn_readfirstlane(w.w)};
  };

  const uint32_t rowbytes = (uint32_t)L * Q * 4;
  const uint32_t treebytes = (uint32_t)ni * rowbytes;
  const rsrc_t rdp = make_rsrc(A.dp + (size_t)tree * ni * L * Q, treebytes);
  constexpr bool keep_s = FWD && BWD && KS;
  const rsrc_t rsr = make_rsrc(keep_s ? A.srow + (size_t)tree * ni * L * Q : A.dp, treebytes);
  const int tb = tile * kWave * Q * 4;
  const int tbytes = (min(L, (tile + 1) * kWave) - tile * kWave) * Q * 4;
  // row store through the pair's scratch: both halves' values of the 64
  // sites laid out [site][Q] (each wave writes its 10 states), then the
  // tile's contiguous row block goes out in 16-B pieces split between the
  // two waves (lane l of wave h: pieces 64 h + l + 128 t), every wave
  // instruction 1 KiB contiguous (sankoff_site.hip store_row)
  auto store_row = [&](rsrc_t r, int row, const float (&v)[kH]) {
    pair_sync();  // the partner is done reading xr
    if (QC == kSQ2) {
      // 8-byte aligned pairs (Q and s0 even)
#pragma unroll
      for (int k = 0; k < kH; k += 2)
        *reinterpret_cast<float2*>(xr + lane * Q + s0 + k) = make_float2(v[k], v[k + 1]);
    } else {
#pragma unroll
      for (int k = 0; k < kH; ++k)
        if (valid(k)) xr[lane * Q + s0 + k] = v[k];
    }
    pair_sync();
    const int npieces = Q * kWave * 4 / 16;  // Q * 16
    const bool q4 = (Q & 3) == 0;
    if (q4) {
      u32x4 w[3];
      int o[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int pc = kWave * hf + lane + 2 * kWave * t;
        o[t] = pc < npieces ? 16 * pc : -1;
        w[t] = o[t] >= 0 ? *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(xr) + o[t])
                         : u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int t = 0; t < 3; ++t)
        if (o[t] >= 0)
          __builtin_amdgcn_raw_buffer_store_b128(w[t], r, o[t] < tbytes ? tb + o[t] : 0x7FFFFFF0,
                                                 row * rowbytes, 0);
      // gfx950 store-data hazard: one wait state after the
      // stores, their data registers held through it
      asm volatile("s_nop 0" ::: "memory");
#pragma unroll
      for (int t = 0; t < 3; ++t) asm volatile("" ::"v"(w[t]));
    } else {
      for (int e = kWave * hf + lane; e < Q * kWave; e += 2 * kWave) {
        const int o = 4 * e;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xr[e]), r, o < tbytes ? tb + o : 0x7FFFFFF0,
                                              row * rowbytes, 0);
      }
    }
  };
  const int vbase = active ? site * Q * 4 : 0x7FFFFFF0;
  // direct (lane-strided) row I/O of this wave's 10 states: at Q = 20 as
  // 16 + 16 + 8 bytes (states 0-3, 4-7, 8-9 | 10-11, 12-15, 16-19; a site's
  // row starts 16-byte aligned): three accesses where 4-byte ones would touch
  // every site's cache line ten times
  auto u4 = [](float a0, float a1, float a2, float a3) {
    return u32x4{__float_as_uint(a0), __float_as_uint(a1), __float_as_uint(a2), __float_as_uint(a3)};
  };
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  auto store_row_direct = [&](rsrc_t r, int row, const float (&v)[kH]) {
    if constexpr (QC == kSQ2) {
      const uint32_t so = row * rowbytes;
      if (hf == 0) {
        const u32x4 w0 = u4(v[0], v[1], v[2], v[3]), w1 = u4(v[4], v[5], v[6], v[7]);
        const u32x2 w2 = u32x2{__float_as_uint(v[8]), __float_as_uint(v[9])};
        __builtin_amdgcn_raw_buffer_store_b128(w0, r, vbase, so, 0);
        __builtin_amdgcn_raw_buffer_store_b128(w1, r, vbase + 16, so, 0);
        __builtin_amdgcn_raw_buffer_store_b64(w2, r, vbase + 32, so, 0);
        // gfx950 store-data hazard
        asm volatile("s_nop 0" ::: "memory");
        asm volatile("" ::"v"(w0), "v"(w1), "v"(w2));
      } else {
        const u32x2 w0 = u32x2{__float_as_uint(v[0]), __float_as_uint(v[1])};
        const u32x4 w1 = u4(v[2], v[3], v[4], v[5]), w2 = u4(v[6], v[7], v[8], v[9]);
        __builtin_amdgcn_raw_buffer_store_b64(w0, r, vbase + 40, so, 0);
        __builtin_amdgcn_raw_buffer_store_b128(w1, r, vbase + 48, so, 0);
        __builtin_amdgcn_raw_buffer_store_b128(w2, r, vbase + 64, so, 0);
        asm volatile("s_nop 0" ::: "memory");
        asm volatile("" ::"v"(w0), "v"(w1), "v"(w2));
      }
    } else {
#pragma unroll
      for (int k = 0; k < kH; ++k)
        if (valid(k))
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[k]), r, vbase + 4 * (s0 + k),
                                                row * rowbytes, 0);
    }
  };
  auto load_row_r = [&](rsrc_t rr, int row, float (&v)[kH]) {
    if constexpr (QC == kSQ2) {
      const uint32_t so = row * rowbytes;
      u32x4 a, b;
      u32x2 c;
      if (hf == 0) {
        a = __builtin_amdgcn_raw_buffer_load_b128(rr, vbase, so, 1);
        b = __builtin_amdgcn_raw_buffer_load_b128(rr, vbase + 16, so, 1);
        c = __builtin_amdgcn_raw_buffer_load_b64(rr, vbase + 32, so, 1);
        const uint32_t x[kH] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y};
#pragma unroll
        for (int k = 0; k < kH; ++k) v[k] = __uint_as_float(x[k]);
      } else {
        c = __builtin_amdgcn_raw_buffer_load_b64(rr, vbase + 40, so, 1);
        a = __builtin_amdgcn_raw_buffer_load_b128(rr, vbase + 48, so, 1);
        b = __builtin_amdgcn_raw_buffer_load_b128(rr, vbase + 64, so, 1);
        const uint32_t x[kH] = {c.x, c.y, a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < kH; ++k) v[k] = __uint_as_float(x[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kH; ++k)
        v[k] = valid(k) ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, vbase + 4 * (s0 + k),
                                                                               row * rowbytes, 1))
                        : 0.0f;
    }
  };
  auto load_row = [&](int row, float (&v)[kH]) { load_row_r(rdp, row, v); };
  auto slot_get = [&](int sl, float (&v)[kH]) {
#pragma unroll
    for (int k = 0; k < kH; ++k) v[k] = slots[(size_t)sl * kSlotF2 + (s0 + k) * kWave + lane];
  };
  auto slot_put = [&](int sl, const float (&v)[kH]) {
#pragma unroll
    for (int k = 0; k < kH; ++k) slots[(size_t)sl * kSlotF2 + (s0 + k) * kWave + lane] = v[k];
  };
  auto tab_row = [&](int code, float (&m)[kH]) {
#pragma unroll
    for (int c = 0; c < kH / 2; ++c) {
      const float2 w = reinterpret_cast<const float2*>(tab + code * kSQ2 + s0)[c];
      m[2 * c] = w.x;
      m[2 * c + 1] = w.y;
    }
  };
  auto leaf_code = [&](int desc) -> int {
    return ((desc >> 24) & 3) == kKindLeaf ? (int)lleaf[(desc & 0xFFFF) * kWave + lane] : Q;
  };
  const float* tmg = A.ptab;
  const float* tsg = A.ptab + kSitePairs * kSQ2;
  auto pair_of = [&](const I4& e) -> int { return site_pair(leaf_code(e.y), leaf_code(e.z)); };
  auto load_tab = [&](const float* t, int p, float (&v)[kH]) {
    const float2* r = reinterpret_cast<const float2*>(t + p * kSQ2 + s0);
#pragma unroll
    for (int c = 0; c < kH / 2; ++c) {
      const float2 w = r[c];
      v[2 * c] = w.x;
      v[2 * c + 1] = w.y;
    }
  };

  // softmin weights of a child with D = d (both halves): md = min_j D_j over
  // the pair, u_j = exp2((md - D_j) a) for this wave's j
  auto weights_u = [&](const float (&d)[kH], float& md, float (&u)[kH]) {
    float m0 = d[0];
#pragma unroll
    for (int k = 1; k < kH; ++k) m0 = valid(k) ? fminf(m0, d[k]) : m0;
    if (!valid(0)) m0 = INFINITY;
    md = fminf(m0, exchange(m0));
    const float mda = md * a;
#pragma unroll
    for (int k = 0; k < kH; ++k) u[k] = valid(k) ? fast_exp2(fmaf(-d[k], a, mda)) : 0.0f;
  };
  // ... and s_i = sum_j K_ij u_j for this wave's i, j over the whole site in
  // the original order (u of both halves through the pair's xu rows)
  auto weights = [&](const float (&d)[kH], float& md, float (&u)[kH], float (&s)[kH]) {
    weights_u(d, md, u);
#pragma unroll
    for (int k = 0; k < kH; ++k) xu[(s0 + k) * kWave + lane] = u[k];
    pair_sync();
    f2 s2[kH / 2];
#pragma unroll
    for (int k = 0; k < kH / 2; ++k) s2[k] = pk(0.0f, 0.0f);
    const cptr<float> KT = K + kSQ2 * kSQ2 + s0;
#pragma unroll 2
    for (int j = 0; j < Q; ++j) {
      const cptr<float> kc = KT + j * kSQ2;
      const float uj = xu[j * kWave + lane];
#pragma unroll
      for (int k = 0; k < kH; k += 2) s2[k / 2] = __builtin_elementwise_fma(pk(kc[k], kc[k + 1]), pk(uj, uj), s2[k / 2]);
    }
#pragma unroll
    for (int k = 0; k < kH; k += 2) {
      s[k] = valid(k) ? s2[k / 2].x : 1.0f;
      s[k + 1] = valid(k + 1) ? s2[k / 2].y : 1.0f;
    }
  };
  auto message_add = [&](const float (&d)[kH], float (&dv)[kH], bool first, int srow_row = -1) {
    float md, u[kH], s[kH];
    weights(d, md, u, s);
    if (keep_s && srow_row >= 0) store_row(rsr, srow_row, s);
    const float base = md + cmin;
#pragma unroll
    for (int k = 0; k < kH; ++k) {
      const float m = valid(k) ? fmaf(-bcoef, fast_log2(s[k]), base) : 0.0f;
      dv[k] = first ? m : dv[k] + m;
    }
  };
  auto leaf_add = [&](int desc, float (&dv)[kH], bool first) {
    float m[kH];
    tab_row(leaf_code(desc), m);
#pragma unroll
    for (int k = 0; k < kH; ++k) dv[k] = first ? m[k] : dv[k] + m[k];
  };
  auto cheap_d = [&](const I4& e, float (&d)[kH]) {
    leaf_add(e.y, d, true);
    leaf_add(e.z, d, false);
  };
  auto cherry_add = [&](const I4& e, float (&dv)[kH], bool first, bool store) {
    float m[kH];
    load_tab(tmg, pair_of(e), m);
    if (store) {
      float d[kH];
      cheap_d(e, d);
      store_row(rdp, e.x, d);
    }
#pragma unroll
    for (int k = 0; k < kH; ++k) dv[k] = first ? m[k] : dv[k] + m[k];
  };
  auto inline_d = [&](int idx, float (&d)[kH], bool store) {
    const I4 e = load_step(inl, idx);
    if (e.w <= 1) {
      cheap_d(e, d);
    } else {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int desc = c == 0 ? e.y : e.z;
        if (((desc >> 24) & 3) == kKindInline) {
          cherry_add(load_step(inl, desc & 0xFFFF), d, c == 0, store);
        } else {
          leaf_add(desc, d, c == 0);
        }
      }
    }
    if (store) store_row(rdp, e.x, d);
  };
  auto child_add = [&](int desc, float (&dv)[kH], bool first, bool store) {
    const int kind = (desc >> 24) & 3;
    if (kind == kKindInt) {
      float d[kH];
      slot_get((desc >> 16) & 0xFF, d);
      message_add(d, dv, first, desc & 0xFFFF);
    } else if (kind == kKindInline) {
      const I4 e = load_step(inl, desc & 0xFFFF);
      if (e.w <= 1) {
        cherry_add(e, dv, first, store);
      } else {
        float d[kH];
        inline_d(desc & 0xFFFF, d, store);
        message_add(d, dv, first, e.x);
      }
    } else {
      leaf_add(desc, dv, first);
    }
  };

  // ---- forward: stage by stage, a stage's tasks round-robin over the pairs ----
  if constexpr (FWD) {
    for (int s = 0; s < S; ++s) {
      const int lo = pword(4 + s), hi = pword(5 + s);
      const bool split = 2 * (hi - lo) <= kPairs;
      const int nit = split ? 2 * (hi - lo) : hi - lo;
      I4 stp = I4{0, 0, 0, 0};
      float dv[kH];
      for (int it = pr; it < nit; it += kPairs) {
        stp = load_step(steps, lo + (split ? it >> 1 : it));
        const int c_lo = split ? (it & 1) : 0, c_hi = split ? c_lo + 1 : 2;
        for (int c = c_lo; c < c_hi; ++c) child_add(c == 0 ? stp.y : stp.z, dv, c == c_lo, true);
        if (split && c_lo == 1) {
          // hand the message over through this pair's xu rows (rows this
          // wave owns; the partner pair reads them after the barrier)
          pair_sync();
#pragma unroll
          for (int k = 0; k < kH; ++k) xu[(s0 + k) * kWave + lane] = dv[k];
        } else if (!split) {
          store_row(rdp, stp.x & 0xFFFF, dv);
          slot_put((stp.x >> 16) & 0xFF, dv);
        }
      }
      if (split) {
        site2_barrier();
        if (pr < nit && (pr & 1) == 0) {
          const float* px = scr + (size_t)(pr + 1) * 2 * kScrF + kScrF;  // pair pr + 1's xu
#pragma unroll
          for (int k = 0; k < kH; ++k) dv[k] = dv[k] + px[(s0 + k) * kWave + lane];
          store_row(rdp, stp.x & 0xFFFF, dv);
          slot_put((stp.x >> 16) & 0xFF, dv);
        }
      }
      site2_barrier();
      SITE2_STAMP(2 + (s < 5 ? s : 5));
    }
  }

  // ---- root (the last stage's only task): wave 0 computes it from the
  // whole D vector in its slot -- the one-wave arithmetic of
  // sankoff_site.hip, so score and cotangent are bitwise that kernel's ----
  const int root_slot = (load_step(steps, pword(4 + S - 1)).x >> 16) & 0xFF;
  if (wv == 0) {
    float droot[kSQ2], groot[kSQ2];
    if constexpr (FWD) {
#pragma unroll
      for (int i = 0; i < kSQ2; ++i) droot[i] = slots[(size_t)root_slot * kSlotF2 + i * kWave + lane];
    } else {
      const int vb = active ? site * Q * 4 : 0x7FFFFFF0;
#pragma unroll
      for (int i = 0; i < kSQ2; ++i)
        droot[i] = i < Q ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rdp, vb + 4 * i,
                                                                                (ni - 1) * rowbytes, 1))
                         : 0.0f;
    }
    float mn = droot[0];
#pragma unroll
    for (int i = 1; i < kSQ2; ++i) mn = i < Q ? fminf(mn, droot[i]) : mn;
    float score;
    if (A.hard_root) {
      float cnt = 0.0f;
#pragma unroll
      for (int i = 0; i < kSQ2; ++i) cnt += (i < Q && droot[i] == mn) ? 1.0f : 0.0f;
      const float r = 1.0f / cnt;
#pragma unroll
      for (int i = 0; i < kSQ2; ++i) groot[i] = (i < Q && droot[i] == mn) ? r : 0.0f;
      score = mn;
    } else {
      float ls = 0.0f, lt = 0.0f;
#pragma unroll
      for (int i = 0; i < kSQ2; ++i) {
        groot[i] = i < Q ? fast_exp2((mn - droot[i]) * a) : 0.0f;
        const bool tie = i < Q && droot[i] == mn;
        ls += tie ? 0.0f : groot[i];
        lt += tie ? 1.0f : 0.0f;
      }
      const float sum = lt + ls;
      const float rs = __builtin_amdgcn_rcpf(sum);
#pragma unroll
      for (int i = 0; i < kSQ2; ++i) groot[i] *= rs;
      score = fmaf(-bcoef, fast_log2(sum), mn);
    }
    if constexpr (FWD) {
      if (active && A.site_score) A.site_score[(size_t)tree * L + site] = score;
      const double tot = wave_sum_lane0(active ? (double)score : 0.0);
      if (lane == 0) A.part_tree[blockIdx.x] = tot;
    }
    const float f = active ? (A.dts ? as_const(A.dts)[tree] : 1.0f) : 0.0f;
#pragma unroll
    for (int i = 0; i < kSQ2; ++i) groot[i] *= f;
    if constexpr (BWD) {
#pragma unroll
      for (int i = 0; i < kSQ2; ++i) slots[(size_t)root_slot * kSlotF2 + i * kWave + lane] = groot[i];
    }
  }

  if constexpr (BWD) {
    SITE2_STAMP(8);
    if constexpr (FWD) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    SITE2_STAMP(9);
    // dC accumulators on v_mfma_f32_16x16x32_bf16, split by rows between
    // the pair: wave hf owns parent states i in [16 hf, 16 hf + 16) (rows
    // >= 20 discarded) over all 64 sites, two 16-column tiles (j < 32);
    // acc1 = sum r u^T (x K at the end), acc2 = the leaf one-hot terms.
    // 16 accumulator VGPRs instead of 32 (128-VGPR budget: 4 waves / SIMD)
    f4 acc1[2], acc2[2];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc1[c][r] = 0.0f;
        acc2[c][r] = 0.0f;
      }
    const int l16 = lane & 15, kq = lane >> 4;  // operand row / column; k group (8 sites)
    const int arow = 16 * hf + l16 < kSQ2 ? 16 * hf + l16 : 0;  // rows >= 20: any finite data
    const int bcol0 = l16, bcol1 = 16 + l16 < kSQ2 ? 16 + l16 : 0;
    auto mf = [&](const u32x4& x, const u32x4& y, f4& c) {
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v, x), __builtin_bit_cast(bf16x8v, y),
                                                  c, 0, 0, 0);
    };
    // acc1 += (xr)(xu)^T: r and u split exactly into three truncated bf16
    // pieces (sankoff_site.hip), the six products down to 2^-16, k = 32 sites
    auto outer_mfma = [&]() {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        asm volatile("" ::: "memory");  // one k-step's pieces live at a time
        const int sg = 32 * ks + 8 * kq;
        u32x4 ah, am, al;
        split3p(xr + swz2(arow, sg), xr + swz2(arow, sg + 4), ah, am, al);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int bc = c == 0 ? bcol0 : bcol1;
          u32x4 bh, bm, bl;
          split3p(xu + swz2(bc, sg), xu + swz2(bc, sg + 4), bh, bm, bl);
          mf(ah, bl, acc1[c]);
          mf(al, bh, acc1[c]);
          mf(am, bm, acc1[c]);
          mf(am, bh, acc1[c]);
          mf(ah, bm, acc1[c]);
          mf(ah, bh, acc1[c]);
        }
      }
    };
    auto outer = [&](const float (&r)[kH], const float (&u)[kH]) {
      pair_sync();  // the partner is done with xr / xu
#pragma unroll
      for (int k = 0; k < kH; ++k) {
        xr[swz2(s0 + k, lane)] = r[k];
        xu[swz2(s0 + k, lane)] = u[k];
      }
      pair_sync();
      outer_mfma();
    };
    // acc2 += g (the leaf children's one-hot counts)^T: g in three bf16
    // pieces against exact 0 / 1 / 2 counts
    auto leaf_hist = [&](const float (&g)[kH], int d0, int d1) {
      pair_sync();
#pragma unroll
      for (int k = 0; k < kH; ++k) xr[swz2(s0 + k, lane)] = g[k];
      pair_sync();
      const bool l0 = ((d0 >> 24) & 3) == kKindLeaf, l1 = ((d1 >> 24) & 3) == kKindLeaf;
      const uint32_t* c0 = reinterpret_cast<const uint32_t*>(lleaf + (d0 & 0xFFFF) * kWave);
      const uint32_t* c1 = reinterpret_cast<const uint32_t*>(lleaf + (d1 & 0xFFFF) * kWave);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        asm volatile("" ::: "memory");
        const int sg = 32 * ks + 8 * kq;
        u32x4 ph, pm, pl;
        split3p(xr + swz2(arow, sg), xr + swz2(arow, sg + 4), ph, pm, pl);
        const uint32_t w0[2] = {l0 ? c0[sg >> 2] : 0xFFFFFFFFu, l0 ? c0[(sg >> 2) + 1] : 0xFFFFFFFFu};
        const uint32_t w1[2] = {l1 ? c1[sg >> 2] : 0xFFFFFFFFu, l1 ? c1[(sg >> 2) + 1] : 0xFFFFFFFFu};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const uint32_t col = 16 * c + l16;
          u32x4 pb;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t bb[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int si = 2 * q + e;
              const uint32_t a0 = (w0[si >> 2] >> (8 * (si & 3))) & 0xFF, a1 = (w1[si >> 2] >> (8 * (si & 3))) & 0xFF;
              const int cnt = (a0 == col ? 1 : 0) + (a1 == col ? 1 : 0);
              bb[e] = cnt == 0 ? 0u : cnt == 1 ? 0x3F80u : 0x4000u;  // bf16 0, 1, 2
            }
            pb[q] = bb[0] | (bb[1] << 16);
          }
          mf(ph, pb, acc2[c]);
          mf(pm, pb, acc2[c]);
          mf(pl, pb, acc2[c]);
        }
      }
    };
    // adjoint of one internal child given u (this wave's j) and s (this
    // wave's i): r_i = g_i / s_i; t_j = sum_i K_ij r_i over the whole site
    // (r of both halves through the pair's xr rows, the original order);
    // gc_j = u_j t_j; dC += r u^T (this wave's sites)
    auto child_adj_rest = [&](const float (&u)[kH], float (&r)[kH], const float (&g)[kH],
                              float (&gc)[kH]) {
#pragma unroll
      for (int k = 0; k < kH; ++k) r[k] = valid(k) ? g[k] * __builtin_amdgcn_rcpf(r[k]) : 0.0f;
      pair_sync();
#pragma unroll
      for (int k = 0; k < kH; ++k) {
        xr[swz2(s0 + k, lane)] = r[k];
        xu[swz2(s0 + k, lane)] = u[k];
      }
      pair_sync();
      f2 t2[kH / 2];
#pragma unroll
      for (int k = 0; k < kH / 2; ++k) t2[k] = pk(0.0f, 0.0f);
#pragma unroll 2
      for (int i = 0; i < Q; ++i) {
        const cptr<float> kr = K + i * kSQ2 + s0;
        const float ri = xr[swz2(i, lane)];
#pragma unroll
        for (int k = 0; k < kH; k += 2)
          t2[k / 2] = __builtin_elementwise_fma(pk(kr[k], kr[k + 1]), pk(ri, ri), t2[k / 2]);
      }
#pragma unroll
      for (int k = 0; k < kH; k += 2) {
        gc[k] = u[k] * t2[k / 2].x;
        gc[k + 1] = u[k + 1] * t2[k / 2].y;
      }
      outer_mfma();
    };
    auto child_adj = [&](const float (&d)[kH], const float (&g)[kH], float (&gc)[kH]) {
      float md, u[kH], r[kH];
      weights(d, md, u, r);
      child_adj_rest(u, r, g, gc);
    };
    auto cherry_adj = [&](const I4& e, const float (&d)[kH], const float (&g)[kH], float (&gc)[kH]) {
      float md, u[kH], r[kH];
      load_tab(tsg, pair_of(e), r);
      weights_u(d, md, u);
      child_adj_rest(u, r, g, gc);
    };
    auto sent_adj = [&](const float (&g)[kH]) {
      float r[kH], u[kH];
#pragma unroll
      for (int k = 0; k < kH; ++k) {
        r[k] = g[k] * sinv[s0 + k];
        u[k] = valid(k) ? 1.0f : 0.0f;
      }
      outer(r, u);
    };
    const bool want_marg = A.marg != nullptr;
    const rsrc_t rmg = make_rsrc(want_marg ? A.marg + (size_t)tree * ni * L * Q : A.dp, treebytes);
    int8_t* at = A.anc ? A.anc + (size_t)tree * ni * L + site : nullptr;
    auto emit = [&](int row, const float (&g)[kH]) {
      if (want_marg) store_row_direct(rmg, row, g);
      if (at) {
        // first index of the maximum over the site (sankoff_site.hip emit):
        // each half's best, then the lower half wins ties
        float bv = g[0];
        int bi = s0;
#pragma unroll
        for (int k = 1; k < kH; ++k)
          if (valid(k) && g[k] > bv) {
            bv = g[k];
            bi = s0 + k;
          }
        if (!valid(0)) bv = -INFINITY;
        const float ov = exchange(bv);
        const int oi = __float_as_int(exchange(__int_as_float(bi)));
        if (hf == 0 && active) at[(size_t)row * L] = (int8_t)(ov > bv ? oi : bi);
      }
    };
    auto leafish_adj = [&](const float (&g)[kH], int d0, int d1) {
      const int k0 = (d0 >> 24) & 3, k1 = (d1 >> 24) & 3;
      if (k0 == kKindLeaf || k1 == kKindLeaf) {
        leaf_hist(g, d0, d1);
        const int nmiss = (k0 == kKindLeaf && leaf_code(d0) == Q ? 1 : 0) +
                          (k1 == kKindLeaf && leaf_code(d1) == Q ? 1 : 0);
        if (__any(active && nmiss != 0)) {
          const float fm = active ? (float)nmiss : 0.0f;
          float r[kH], u[kH];
#pragma unroll
          for (int k = 0; k < kH; ++k) {
            r[k] = fm * (g[k] * sinv[s0 + k]);
            u[k] = valid(k) ? 1.0f : 0.0f;
          }
          outer(r, u);
        }
      }
      if (k0 == 0) sent_adj(g);
      if (k1 == 0) sent_adj(g);
    };
    auto inline_adj = [&](int idx, const float (&g)[kH]) {
      const I4 e = load_step(inl, idx);
      emit(e.x, g);
      if (e.w > 1) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? e.y : e.z;
          if (((desc >> 24) & 3) == kKindInline) {
            const I4 e2 = load_step(inl, desc & 0xFFFF);
            float dc[kH], gc[kH];
            cheap_d(e2, dc);
            cherry_adj(e2, dc, g, gc);
            emit(e2.x, gc);
            leafish_adj(gc, e2.y, e2.z);
          }
        }
      }
      leafish_adj(g, ((e.y >> 24) & 3) == kKindInline ? (int)0x7F000000 : e.y,
                  ((e.z >> 24) & 3) == kKindInline ? (int)0x7F000000 : e.z);
    };
    auto adj_task = [&](const I4& stp, int c_lo, int c_hi) {
      const int vslot = (stp.x >> 16) & 0xFF;
      int lf0 = 0x7F000000, lf1 = 0x7F000000;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if (c < c_lo || c >= c_hi) continue;
        const int desc = c == 0 ? stp.y : stp.z;
        const int kind = (desc >> 24) & 3;
        if (kind == kKindInt || kind == kKindInline) {
          const I4 ie = kind == kKindInline ? load_step(inl, desc & 0xFFFF) : I4{desc & 0xFFFF, 0, 0, 2};
          float d[kH], g[kH], gc[kH];
          if (ie.w > 1 && keep_s) {
            float sv[kH], md, u[kH];
            load_row(ie.x, d);
            weights_u(d, md, u);
            load_row_r(rsr, ie.x, sv);
#pragma unroll
            for (int k = 0; k < kH; ++k) sv[k] = active ? sv[k] : 1.0f;
            slot_get(vslot, g);
            if (c == 0) emit(stp.x & 0xFFFF, g);
            child_adj_rest(u, sv, g, gc);
          } else {
            if (ie.w > 1)
              load_row(ie.x, d);
            else
              cheap_d(ie, d);
            slot_get(vslot, g);
            if (c == 0) emit(stp.x & 0xFFFF, g);
            if (ie.w > 1)
              child_adj(d, g, gc);
            else
              cherry_adj(ie, d, g, gc);
          }
          if (kind == kKindInt)
            slot_put((desc >> 16) & 0xFF, gc);
          else
            inline_adj(desc & 0xFFFF, gc);
        } else if (c == 0) {
          lf0 = desc;
          float g[kH];
          slot_get(vslot, g);
          emit(stp.x & 0xFFFF, g);
        } else {
          lf1 = desc;
        }
      }
      if (lf0 != 0x7F000000 || lf1 != 0x7F000000) {
        float g[kH];
        slot_get(vslot, g);
        leafish_adj(g, lf0, lf1);
      }
    };
    for (int s = S - 1; s >= 0; --s) {
      const int lo = pword(4 + s), hi = pword(5 + s);
      const bool split = 2 * (hi - lo) <= kPairs;
      const int nit = split ? 2 * (hi - lo) : hi - lo;
      for (int it = pr; it < nit; it += kPairs) {
        const int c_lo = split ? (it & 1) : 0;
        adj_task(load_step(steps, lo + (split ? it >> 1 : it)), c_lo, split ? c_lo + 1 : 2);
      }
      site2_barrier();
      SITE2_STAMP(10 + (S - 1 - s < 5 ? S - 1 - s : 5));
    }

    // ---- dC partial: dC_ij = K_ij acc1_ij + acc2_ij per pair, the 8 pairs
    // summed in order through LDS (slots / scratch are dead) ----
    double* red = reinterpret_cast<double*>(scr);  // [pairs][Q][Q] (<= 26 KB)
    const int Q2 = Q * Q;
    // wave hf's rows; rows of the partner's range are zero in this wave's
    // slice (each (i, j) written by the one wave that owns row i)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * hf + 4 * kq + r, j = 16 * c + l16;
        if (i < Q && j < Q)
          red[(size_t)pr * Q2 + i * Q + j] = (double)acc1[c][r] * (double)K[i * kSQ2 + j] + (double)acc2[c][r];
      }
    __syncthreads();
    const int nb = A.B * A.tiles;
    for (int e = threadIdx.x; e < Q2; e += kSW2 * kWave) {
      double tsum = red[e];
#pragma unroll
      for (int w = 1; w < kPairs; ++w) tsum += red[(size_t)w * Q2 + e];
      A.part_dc[(size_t)e * nb + blockIdx.x] = tsum;
    }
    SITE2_STAMP(16);
  }
}

}  // namespace

size_t site2_lds_bytes(int np, int n_slots, int nl, int ni) {
  const size_t b = ((size_t)n_slots * kSlotF2 + (size_t)np * 2 * kScrF + 2 * np * 2 * kWave + 16 + kTabF2 +
                    lp_tree_ints(ni)) * 4 +
                   (size_t)nl * kWave;
  return (b + 15) & ~(size_t)15;
}

// TREX_SITE2 (read per call): "1" the largest pair count whose LDS fits
// (8, 6, 4), "8" / "6" / "4" that one (when it fits); unset / "0": the
// one-wave kernel (sankoff_site.hip)
static int site2_pairs(int lp_slots, int nl, int ni) {
  const char* e = std::getenv("TREX_SITE2");
  if (!e || e[0] < '1' || e[0] > '9') return 0;
  const int want = e[0] == '1' ? 0 : e[0] - '0';
  for (int np : {8, 6, 4})
    if ((want == 0 || want == np) && site2_lds_bytes(np, lp_slots, nl, ni) <= 160 * 1024) return np;
  return 0;
}

bool site2_on(int lp_slots, int nl, int ni) { return site2_pairs(lp_slots, nl, ni) > 0; }

static int g_site2_launches = 0;  // host-side count (tests: the pair kernel did run)

int site2_run(const char* fn, const WideCall& c, const int32_t* lanes, int lp_slots,
              const int* flag, const float* kg) {
  const int np = site2_pairs(lp_slots, c.nl, c.ni);
  if (np == 0) return set_error(TREX_E_ARG, "%s: the wave-pair kernel does not fit", fn);
  const int tiles = site_tiles(c.L);
  const size_t lds = site2_lds_bytes(np, lp_slots, c.nl, c.ni);
  if ((int64_t)c.B * tiles > 0x7FFFFFFF) return set_error(TREX_E_ARG, "%s: grid too large", fn);
  hipStream_t st = (hipStream_t)c.stream;
  Site2Args A;
  A.lanes = lanes;
  A.stride = lp_tree_ints(c.ni);
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
  A.kg = kg;
  A.ptab = kg - kSiteTabBytes / 4;
  A.srow = c.phase == 3 ? c.site_srow : nullptr;
  A.flag = flag;
  A.n_slots = lp_slots;
  auto go = [&](auto kernel, int npairs) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kernel, dim3((int)nb), dim3(2 * npairs * kWave), lds, st, A);
  };
  auto pick = [&](auto np_c) {
    constexpr int NP = decltype(np_c)::value;
    const bool ks = A.srow != nullptr;
    if (c.Q == kSQ2) {
      if (c.phase == 1)
        go(sankoff_site2_kernel<1, kSQ2, false, NP>, NP);
      else if (c.phase == 2)
        go(sankoff_site2_kernel<2, kSQ2, false, NP>, NP);
      else if (ks)
        go(sankoff_site2_kernel<3, kSQ2, true, NP>, NP);
      else
        go(sankoff_site2_kernel<3, kSQ2, false, NP>, NP);
    } else {
      if (c.phase == 1)
        go(sankoff_site2_kernel<1, 0, false, NP>, NP);
      else if (c.phase == 2)
        go(sankoff_site2_kernel<2, 0, false, NP>, NP);
      else if (ks)
        go(sankoff_site2_kernel<3, 0, true, NP>, NP);
      else
        go(sankoff_site2_kernel<3, 0, false, NP>, NP);
    }
  };
  if (np == 8)
    pick(std::integral_constant<int, 8>());
  else if (np == 6)
    pick(std::integral_constant<int, 6>());
  else
    pick(std::integral_constant<int, 4>());
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  ++g_site2_launches;
  return TREX_OK;
}

}  // namespace trex

#ifdef TREX_SITE2_TIMING
extern "C" int trex_debug_site2_times(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(trex::g_site2_t), sizeof(trex::g_site2_t)) == hipSuccess ? 0 : -4;
}
#endif

// launches of the wave-pair kernel so far (tests check that TREX_SITE2 took effect)
extern "C" int trex_debug_site2_launches(void) { return trex::g_site2_launches; }
