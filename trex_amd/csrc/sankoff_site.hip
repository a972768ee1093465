// libtrexhip.so -- lane-per-site Sankoff kernel for the factored softmin,
// 4 < Q <= 20 states (C3: protein, Q = 20), gfx950.
//
// Same semantics as sankoff_wide.hip (trex src/trex/sankoff.py run_dp
// :24-94, run_sankoff :114-188, the build-defined softmin adjoint) for the
// factored softmin (K = exp(-(C - cmin) / tau), range(C) / tau <= 40) with
// exact leaf messages.  The state-parallel kernel, launched first, decides
// the mode from the cost matrix on the device (every workgroup; it exits
// when this kernel takes the call, and serves every other mode) and its
// workgroup 0 writes K, K^T and a flag into the workspace (wide_dev.h
// site_gate_write); this kernel exits unless the flag is set, and the
// partial reduce picks this kernel's tiles.
//
// Mapping.  A work item is one tree x 64 sites, a workgroup of 8 waves; lane
// = site, a lane keeps all Q states of a vector in registers.  The per-site
// state x state work is then lane-local:
//   s = K u   (forward message, adjoint weights; sankoff.py:67-68)
//   t = K^T r (child cotangent)
// as packed-FP32 FMAs with K read by scalar loads -- every lane of the wave
// uses the same K, so it costs no VGPRs and no LDS bandwidth.  The one
// cross-site reduction, dC = sum over sites and children of r u^T (x K), runs
// on the matrix core: per child the wave writes r and u to its LDS scratch,
// reads them back transposed and issues 32 v_mfma_f32_32x32x2_f32 (k = two
// sites each); leaf children add g e_code^T into a second accumulator the
// same way (the one-hot columns built from the leaf codes).
//
// The tree runs as the height-levelled task program of plan.cpp
// (lane_program_one_tree): rows of height <= 2 are recomputed inline by the
// task that consumes them (their D from the leaf message table, their
// cotangent passed in registers), every other row is a task whose D (forward)
// and cotangent (adjoint) live in an interval-coloured LDS slot; a stage's
// tasks are dealt round-robin to the waves, an LDS barrier between stages.
// The adjoint re-reads task rows' D from the HBM DP table (the roofline's
// re-read) and recomputes inline rows' D from the leaves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "sankoff_dev.h"
#include "trex_common.h"
#include "wide_dev.h"

namespace trex {

#ifndef TREX_SITE_LOAD_AUX
#define TREX_SITE_LOAD_AUX 1  // cache policy of the adjoint's DP-row re-reads (1 = sc0)
#endif
namespace {
constexpr int kSiteLoadAux = TREX_SITE_LOAD_AUX;

constexpr int kSQ = kSiteSQ;               // states per lane (Q padded to 20)
constexpr int kSWv = 8;                    // waves per workgroup
constexpr int kSlotF = kSQ * kWave;        // floats per slot / scratch vector
constexpr int kTabF = (kSQ + 1) * kSQ + kSQ;  // leaf messages T[Q + 1][kSQ] + 1 / sum_j K_ij

typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifndef SITE_DC_BF16
#define SITE_DC_BF16 1  // 0: the dC outer products on f32 32x32x2 MFMAs (A/B, PERFLOG)
#endif

// eight floats (two float4 at p0, p1) split exactly into truncated bf16
// pieces x = h + m + l, packed two per dword in k order
__device__ __forceinline__ void split3(const float* p0, const float* p1, u32x4& h, u32x4& m, u32x4& l) {
  const float4 a = *reinterpret_cast<const float4*>(p0), b = *reinterpret_cast<const float4*>(p1);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // the two residual subtractions of a pair as one v_pk_add_f32 each
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const f2 x = pk(v[2 * q], v[2 * q + 1]);
    const u2 xb = __builtin_bit_cast(u2, x);
    const f2 r1 = x - __builtin_bit_cast(f2, xb & 0xFFFF0000u);
    const u2 mb = __builtin_bit_cast(u2, r1) & 0xFFFF0000u;
    const u2 lb = __builtin_bit_cast(u2, r1 - __builtin_bit_cast(f2, mb));
    // high halves of (e0, e1) -> one dword, e0 in the low half
    h[q] = __builtin_amdgcn_perm(xb.y, xb.x, 0x07060302u);
    m[q] = __builtin_amdgcn_perm(mb.y, mb.x, 0x07060302u);
    l[q] = __builtin_amdgcn_perm(lb.y, lb.x, 0x07060302u);
  }
}

__device__ __forceinline__ f16v mfma_bf(const u32x4& a, const u32x4& b, const f16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

struct SiteArgs {
  const int* lanes;  // lane programs (trex_common.h)
  int64_t stride;    // ints per tree region
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
  const float* kg;    // K [kSQ][kSQ] and K^T (site_gate_write), zero-padded
  const float* ptab;  // cherry tables TM | TS (site_pair_tables), below K
  int cherry;         // 0: the CH = false variants (TREX_SITE_CHERRY=0, A/B; bitwise the same)
  float* srow;        // fused: s = K u of each computed internal child row, [B][n_int][L][Q]
  const int* flag;    // 1: this kernel handles the launch
  int n_slots;
};

#ifdef TREX_SITE_TIMING
// diagnostic build (tools/build_ab.sh sitet sankoff_site.hip -DTREX_SITE_TIMING):
// lane 0 of every wave of the first 2048 workgroups stamps s_memtime at phase
// boundaries (tools/site_times.py)
__device__ unsigned long long g_site_t[2048][8][20];
#define SITE_STAMP(j)                                                              \
  do {                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 2048 && (j) < 20)                  \
      g_site_t[blockIdx.x][threadIdx.x >> 6][j] = __builtin_amdgcn_s_memtime();   \
  } while (0)
#else
#define SITE_STAMP(j) \
  do {                \
  } while (0)
#endif

__device__ __forceinline__ void site_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// scratch swizzle: row i of a [kSQ][64] scratch keeps site s at s ^ 4 (i & 15)
// (4-site groups stay contiguous; 16 rows read at one site group hit 16
// distinct 16-byte bank groups)
__device__ __forceinline__ int swz(int i, int s) { return i * kWave + (s ^ ((i & 15) << 2)); }

// QC: the alphabet size when it is 20 (C3: every state mask folds away), 0 =
// runtime Q <= 20 with masked padded states
// KS (fused only): keep the forward's s rows for the adjoint (A.srow);
// CH: cherry tables (false: the per-lane mat-vecs, TREX_SITE_CHERRY=0 A/B)
template <int PHASE, int QC, bool KS = false, bool CH = true>
__global__ __launch_bounds__(kSWv * kWave, 1) void sankoff_site_kernel(SiteArgs A) {
  constexpr bool FWD = (PHASE & 1) != 0;
  constexpr bool BWD = (PHASE & 2) != 0;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (!__builtin_amdgcn_readfirstlane(as_const(A.flag)[0])) return;
  SITE_STAMP(0);
  const int Q = QC ? QC : A.Q;
  const int ni = A.n_int;
  const int L = A.L;
  const int tree = blockIdx.x / A.tiles;
  const int tile = blockIdx.x - tree * A.tiles;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x % kWave;
  const int site = tile * kWave + lane;
  const bool active = site < L;
  const float a = A.a, bcoef = A.bcoef;
  const cptr<float> K = as_const(A.kg);

  // ---- LDS: slots [n_slots][kSQ][64] | scratch [kSWv][2][kSQ][64] | T, sinv | leaf codes ----
  float* slots = lds;
  float* scr = slots + (size_t)A.n_slots * kSlotF;
  float* xr = scr + (size_t)wv * 2 * kSlotF;
  float* xu = xr + kSlotF;
  float* tab = scr + (size_t)kSWv * 2 * kSlotF;
  float* sinv = tab + (kSQ + 1) * kSQ;
  int* lprog = reinterpret_cast<int*>(tab + kTabF);  // this tree's lane program
  const int pints = (int)A.stride;
  int8_t* lleaf = reinterpret_cast<int8_t*>(lprog + pints);
  // K rows by scalar loads (every lane of the wave uses the same K); the row
  // loops stay rolled (an unrolled product would hoist all Q^2 loads into
  // SGPRs), their per-row results go through the wave's scratch column

  float cmin;
  {
    float lmin = INFINITY;
    for (int e = lane; e < Q * Q; e += kWave) lmin = fminf(lmin, A.cost[e]);
    cmin = uniform(wave_minf(lmin));
  }
  // leaf message table: T[code][i] = C[i][code] (exact: the 1e5 sentinel
  // dominates), T[Q][i] = the all-1e5 row's message, sinv[i] = 1 / sum_j K_ij
  for (int e = threadIdx.x; e < (kSQ + 1) * kSQ; e += kSWv * kWave) {
    const int code = e / kSQ, i = e - code * kSQ;
    float v = 0.0f;
    if (i < Q) {
      if (code < Q) {
        v = A.cost[i * Q + code];
      } else {
        float sk = 0.0f;
        for (int j = 0; j < Q; ++j) sk += A.kg[i * kSQ + j];
        v = fmaf(-bcoef, fast_log2(sk), kSentinel + cmin);
      }
    }
    tab[e] = v;
  }
  if (threadIdx.x < kSQ) {
    const int i = threadIdx.x;
    float sk = 0.0f;
    for (int j = 0; j < Q; ++j) sk += A.kg[i * kSQ + j];
    sinv[i] = i < Q ? __builtin_amdgcn_rcpf(sk) : 0.0f;
  }
  // the tree's program into LDS (one coalesced pass instead of dependent
  // scalar misses on the step chain) and the tile's leaf codes (dwords of 4
  // sites when rows are 4-byte aligned), all loads in flight together
  {
    const int* pg = A.lanes + (size_t)tree * A.stride;
    for (int e = threadIdx.x; e < pints; e += kSWv * kWave) lprog[e] = pg[e];
    const int8_t* lv = A.leaves + (size_t)tree * A.nl * L;
    auto norm = [&](int code) { return ((unsigned)code < (unsigned)Q) ? code : Q; };
    if ((L & 3) == 0) {
      for (int e = threadIdx.x; e < A.nl * (kWave / 4); e += kSWv * kWave) {
        const int leaf = e / (kWave / 4);
        const int s0 = tile * kWave + 4 * (e - leaf * (kWave / 4));
        uint32_t w = 0xFFFFFFFFu;
        if (s0 < L) w = *reinterpret_cast<const uint32_t*>(lv + (size_t)leaf * L + s0);
        uint32_t o = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) o |= (uint32_t)norm((int)(int8_t)(w >> (8 * q))) << (8 * q);
        reinterpret_cast<uint32_t*>(lleaf)[e] = o;
      }
    } else {
      for (int e = threadIdx.x; e < A.nl * kWave; e += kSWv * kWave) {
        const int leaf = e / kWave;
        const int s = tile * kWave + (e - leaf * kWave);
        lleaf[e] = (int8_t)(s < L ? norm((int)lv[(size_t)leaf * L + s]) : Q);
      }
    }
  }
  __syncthreads();
  SITE_STAMP(1);

  // program words from LDS (every lane the same address), made wave-uniform
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
  // fused calls keep each computed child row's s for the adjoint (the
  // forward's mat-vec instead of a second one); srow null: recomputed
  constexpr bool keep_s = FWD && BWD && KS;
  const rsrc_t rsr = make_rsrc(keep_s ? A.srow + (size_t)tree * ni * L * Q : A.dp, treebytes);
  const bool q4 = (Q & 3) == 0;
  // Row I/O through the wave's scratch (xr): a lane's Q values are 4Q
  // bytes apart from its neighbour's in the site-major row, so a direct
  // 16-B-per-lane access touches 5x the cache lines of a contiguous one
  // (C3: a workgroup's forward stage 0 at 45 k cycles of which 21 k were the
  // strided stores; lane-contiguous, 24 k).  The tile's row block (64 sites
  // x Q floats, contiguous in HBM) is instead transposed in LDS: lane l
  // moves bytes [16 (l + 64 c), +16) -- every wave instruction 1 KiB
  // contiguous.  Bytes of sites past L are skipped (stores) / read as 0.
  // the transposes' own ordering point: all of this wave's LDS traffic done
  auto lds_sync = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  const int tb = tile * kWave * Q * 4;  // this tile's first byte in a row
  const int tbytes = (min(L, (tile + 1) * kWave) - tile * kWave) * Q * 4;
  auto store_row = [&](rsrc_t r, int row, const float (&v)[kSQ]) {
#ifdef SITE_DIAG_NOSTORE  // diagnostic: no row stores (wrong results)
    return;
#endif
    if (q4) {
#pragma unroll
      for (int c = 0; c < kSQ / 4; ++c)
        if (4 * c < Q)
          *reinterpret_cast<float4*>(xr + lane * Q + 4 * c) =
              make_float4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
      lds_sync();
      u32x4 w[kSQ / 4];
#pragma unroll
      for (int c = 0; c < kSQ / 4; ++c)
        if (4 * c < Q)
          w[c] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(xr) + 16 * (lane + kWave * c));
#pragma unroll
      for (int c = 0; c < kSQ / 4; ++c) {
        if (4 * c < Q) {
          const int o = 16 * (lane + kWave * c);
          __builtin_amdgcn_raw_buffer_store_b128(w[c], r, o < tbytes ? tb + o : 0x7FFFFFF0, row * rowbytes, 0);
        }
      }
      // gfx950 store-data hazard: a VALU write of a 128-bit store's data VGPR
      // in the instruction right after the store changes the bytes it writes
      // -- also with an SGPR soffset, where LLVM inserts no wait state
      // (tools/micro/store_reuse.hip: 2 % of rows corrupted at distance 1,
      // none after one s_nop).  One wait state after the last
      // store, the data registers held live through it so none is
      // reallocated before it; tests/test_isa_guard_cpu.py checks every
      // code object of the build for the pattern.
      asm volatile("s_nop 0" ::: "memory");
#pragma unroll
      for (int c = 0; c < kSQ / 4; ++c)
        if (4 * c < Q) asm volatile("" ::"v"(w[c]));
    } else {
#pragma unroll
      for (int j = 0; j < kSQ; ++j)
        if (j < Q) xr[lane * Q + j] = v[j];
      lds_sync();
#pragma unroll
      for (int j = 0; j < kSQ; ++j) {
        if (j < Q) {
          const int o = 4 * (lane + kWave * j);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xr[lane + kWave * j]), r,
                                                o < tbytes ? tb + o : 0x7FFFFFF0, row * rowbytes, 0);
        }
      }
    }
    lds_sync();
  };
  // direct (lane-strided) row I/O: the loads stay asynchronous (the wave
  // waits only where it uses the values)
  const int vbase = active ? site * Q * 4 : 0x7FFFFFF0;
  auto store_row_direct = [&](rsrc_t r, int row, const float (&v)[kSQ]) {
    if (q4) {
#pragma unroll
      for (int c = 0; c < kSQ / 4; ++c)
        if (4 * c < Q)
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4{__float_as_uint(v[4 * c]), __float_as_uint(v[4 * c + 1]), __float_as_uint(v[4 * c + 2]),
                    __float_as_uint(v[4 * c + 3])},
              r, vbase + 16 * c, row * rowbytes, 0);
    } else {
#pragma unroll
      for (int j = 0; j < kSQ; ++j)
        if (j < Q) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[j]), r, vbase + 4 * j, row * rowbytes, 0);
    }
  };
  auto load_row_direct = [&](rsrc_t rr, int row, float (&v)[kSQ]) {
    if (q4) {
#pragma unroll
      for (int c = 0; c < kSQ / 4; ++c) {
        u32x4 w = u32x4{0, 0, 0, 0};
        if (4 * c < Q) w = __builtin_amdgcn_raw_buffer_load_b128(rr, vbase + 16 * c, row * rowbytes, kSiteLoadAux);
        v[4 * c] = __uint_as_float(w.x);
        v[4 * c + 1] = __uint_as_float(w.y);
        v[4 * c + 2] = __uint_as_float(w.z);
        v[4 * c + 3] = __uint_as_float(w.w);
      }
    } else {
#pragma unroll
      for (int j = 0; j < kSQ; ++j)
        v[j] = j < Q ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, vbase + 4 * j, row * rowbytes, kSiteLoadAux))
                     : 0.0f;
    }
  };
  auto load_row_t = [&](rsrc_t rr, int row, float (&v)[kSQ]) {
    if (q4) {
#pragma unroll
      for (int c = 0; c < kSQ / 4; ++c) {
        if (4 * c < Q) {
          const int o = 16 * (lane + kWave * c);
          const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rr, o < tbytes ? tb + o : 0x7FFFFFF0,
                                                               row * rowbytes, kSiteLoadAux);
          *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(xr) + o) = w;
        }
      }
      lds_sync();
#pragma unroll
      for (int c = 0; c < kSQ / 4; ++c) {
        float4 w = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (4 * c < Q) w = *reinterpret_cast<const float4*>(xr + lane * Q + 4 * c);
        v[4 * c] = w.x;
        v[4 * c + 1] = w.y;
        v[4 * c + 2] = w.z;
        v[4 * c + 3] = w.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < kSQ; ++j) {
        if (j < Q) {
          const int o = 4 * (lane + kWave * j);
          xr[lane + kWave * j] = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(rr, o < tbytes ? tb + o : 0x7FFFFFF0, row * rowbytes, kSiteLoadAux));
        }
      }
      lds_sync();
#pragma unroll
      for (int j = 0; j < kSQ; ++j) v[j] = j < Q ? xr[lane * Q + j] : 0.0f;
    }
    lds_sync();
  };
#ifndef SITE_LOAD_T
#define SITE_LOAD_T 0  // transposed (synchronous) row loads: slower in the adjoint (PERFLOG)
#endif
  auto load_row_r = [&](rsrc_t rr, int row, float (&v)[kSQ]) {
    if (SITE_LOAD_T)
      load_row_t(rr, row, v);
    else
      load_row_direct(rr, row, v);
  };
  auto load_row = [&](int row, float (&v)[kSQ]) { load_row_r(rdp, row, v); };
#ifdef SITE_DIAG_HOTROW  // diagnostic: the adjoint's row loads all read row 0 (cache-hot; wrong math)
#define SITE_ADJ_ROW(x) 0
#else
#define SITE_ADJ_ROW(x) (x)
#endif
  auto slot_get = [&](int sl, float (&v)[kSQ]) {
#pragma unroll
    for (int j = 0; j < kSQ; ++j) v[j] = slots[(size_t)sl * kSlotF + j * kWave + lane];
  };
  auto slot_put = [&](int sl, const float (&v)[kSQ]) {
#pragma unroll
    for (int j = 0; j < kSQ; ++j) slots[(size_t)sl * kSlotF + j * kWave + lane] = v[j];
  };
  // leaf / sentinel child: its message row of T (code Q = the all-1e5 row)
  auto tab_row = [&](int code, float (&m)[kSQ]) {
#pragma unroll
    for (int c = 0; c < kSQ / 4; ++c) {
      const float4 w = reinterpret_cast<const float4*>(tab + code * kSQ)[c];
      m[4 * c] = w.x;
      m[4 * c + 1] = w.y;
      m[4 * c + 2] = w.z;
      m[4 * c + 3] = w.w;
    }
  };
  auto leaf_code = [&](int desc) -> int {
    return ((desc >> 24) & 3) == kKindLeaf ? (int)lleaf[(desc & 0xFFFF) * kWave + lane] : Q;
  };
  // cherry tables (wide_dev.h site_pair_tables): a height-1 row's forward
  // message (TM) and softmin row sums (TS) by its children's code pair
  const float* tmg = A.ptab;
  const float* tsg = A.ptab + kSitePairs * kSQ;
  auto pair_of = [&](const I4& e) -> int { return site_pair(leaf_code(e.y), leaf_code(e.z)); };
  auto load_tab = [&](const float* t, int p, float (&v)[kSQ]) {
    const float4* r = reinterpret_cast<const float4*>(t + p * kSQ);
#pragma unroll
    for (int c = 0; c < kSQ / 4; ++c) {
      const float4 w = r[c];
      v[4 * c] = w.x;
      v[4 * c + 1] = w.y;
      v[4 * c + 2] = w.z;
      v[4 * c + 3] = w.w;
    }
  };

  // softmin weights of a child with D = d: md = min_j D_j, u_j = exp2((md - D_j) a),
  // s_i = sum_j K_ij u_j (K rows by scalar loads, two partial sums in packed
  // FP32; s_i staged through the wave's scratch, row i at i * 64 + lane)
  auto weights_u = [&](const float (&d)[kSQ], float& md, float (&u)[kSQ]) {
    float m0 = d[0];
#pragma unroll
    for (int j = 1; j < kSQ; ++j) m0 = j < Q ? fminf(m0, d[j]) : m0;
    md = m0;
    const float mda = md * a;
#pragma unroll
    for (int j = 0; j < kSQ; ++j) u[j] = j < Q ? fast_exp2(fmaf(-d[j], a, mda)) : 0.0f;
  };
  auto weights = [&](const float (&d)[kSQ], float& md, float (&u)[kSQ], float (&s)[kSQ]) {
    weights_u(d, md, u);
    // s += K[:, j] u_j over j: independent accumulators (a row-wise dot
    // product would be a chain of dependent FMAs); u_j staged through the
    // scratch, column j of K (= row j of K^T) by scalar loads
#pragma unroll
    for (int j = 0; j < kSQ; ++j) xu[j * kWave + lane] = u[j];
    wave_sync();
    f2 s2[kSQ / 2];
#pragma unroll
    for (int i = 0; i < kSQ / 2; ++i) s2[i] = pk(0.0f, 0.0f);
    const cptr<float> KT = K + kSQ * kSQ;
#pragma unroll 2
    for (int j = 0; j < Q; ++j) {
#ifdef SITE_DIAG_NOSMEM  // diagnostic: one K column for every j (loads hoisted; wrong math)
      const cptr<float> kc = KT;
#else
      const cptr<float> kc = KT + j * kSQ;
#endif
      const float uj = xu[j * kWave + lane];
#pragma unroll
      for (int i = 0; i < kSQ; i += 2) s2[i / 2] = __builtin_elementwise_fma(pk(kc[i], kc[i + 1]), pk(uj, uj), s2[i / 2]);
    }
#pragma unroll
    for (int i = 0; i < kSQ; i += 2) {
      s[i] = i < Q ? s2[i / 2].x : 1.0f;
      s[i + 1] = i + 1 < Q ? s2[i / 2].y : 1.0f;
    }
    wave_sync();
  };
  // message of a child with D = d to every parent state (sankoff.py:67-68, softmin)
  // srow_row >= 0 (fused, keep_s): the child's s row is stored for the adjoint
  auto message_add = [&](const float (&d)[kSQ], float (&dv)[kSQ], bool first, int srow_row = -1) {
    float md, u[kSQ], s[kSQ];
    weights(d, md, u, s);
    if (keep_s && srow_row >= 0) store_row(rsr, srow_row, s);
    const float base = md + cmin;
#pragma unroll
    for (int i = 0; i < kSQ; ++i) {
      const float m = i < Q ? fmaf(-bcoef, fast_log2(s[i]), base) : 0.0f;
      dv[i] = first ? m : dv[i] + m;
    }
  };
  auto leaf_add = [&](int desc, float (&dv)[kSQ], bool first) {
    float m[kSQ];
    tab_row(leaf_code(desc), m);
#pragma unroll
    for (int i = 0; i < kSQ; ++i) dv[i] = first ? m[i] : dv[i] + m[i];
  };
  // D of a height-1 inline row (both children leaves / 1e5 rows): T sums
  auto cheap_d = [&](const I4& e, float (&d)[kSQ]) {
    leaf_add(e.y, d, true);
    leaf_add(e.z, d, false);
  };
  // a cherry's (height-1 row's) message from TM, its D row stored when
  // `store` -- bitwise cheap_d + message_add
  auto cherry_add = [&](const I4& e, float (&dv)[kSQ], bool first, bool store) {
    float m[kSQ];
    load_tab(tmg, pair_of(e), m);
    if (store) {
      float d[kSQ];
      cheap_d(e, d);
      store_row(rdp, e.x, d);
    }
#pragma unroll
    for (int i = 0; i < kSQ; ++i) dv[i] = first ? m[i] : dv[i] + m[i];
  };
  // D of an inline row (height 1 or 2); `store`: write its DP row
  auto inline_d = [&](int idx, float (&d)[kSQ], bool store) {
    const I4 e = load_step(inl, idx);
    if (e.w <= 1) {
      cheap_d(e, d);
    } else {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int desc = c == 0 ? e.y : e.z;
        if (((desc >> 24) & 3) == kKindInline) {
          const I4 e2 = load_step(inl, desc & 0xFFFF);
          if constexpr (CH) {
            cherry_add(e2, d, c == 0, store);
          } else {
            float dc[kSQ];
            cheap_d(e2, dc);
            if (store) store_row(rdp, e2.x, dc);
            message_add(dc, d, c == 0);
          }
        } else {
          leaf_add(desc, d, c == 0);
        }
      }
    }
    if (store) store_row(rdp, e.x, d);
  };
  // a child's contribution to its parent's D
  auto child_add = [&](int desc, float (&dv)[kSQ], bool first, bool store) {
    const int kind = (desc >> 24) & 3;
    if (kind == kKindInt) {
      float d[kSQ];
      slot_get((desc >> 16) & 0xFF, d);
      message_add(d, dv, first, desc & 0xFFFF);
    } else if (kind == kKindInline) {
      const I4 e = load_step(inl, desc & 0xFFFF);
      if (CH && e.w <= 1) {
        cherry_add(e, dv, first, store);
      } else {
        float d[kSQ];
        inline_d(desc & 0xFFFF, d, store);
        message_add(d, dv, first, e.x);
      }
    } else {
      leaf_add(desc, dv, first);
    }
  };

  // ---- forward: stage by stage, a stage's tasks round-robin over the waves ----
  int root_slot = 0;
  if constexpr (FWD) {
    for (int s = 0; s < S; ++s) {
      const int lo = pword(4 + s), hi = pword(5 + s);
      // a stage of at most kSWv / 2 tasks runs one child per wave (items =
      // task x child): the c = 1 wave hands its message over through its
      // scratch column after a barrier, the c = 0 wave adds it (m0 + m1, the
      // one-wave order) and writes the row
      const bool split = 2 * (hi - lo) <= kSWv;
      const int nit = split ? 2 * (hi - lo) : hi - lo;
      I4 stp = I4{0, 0, 0, 0};
      float dv[kSQ];
      for (int it = wv; it < nit; it += kSWv) {
        stp = load_step(steps, lo + (split ? it >> 1 : it));
        const int c_lo = split ? (it & 1) : 0, c_hi = split ? c_lo + 1 : 2;
        for (int c = c_lo; c < c_hi; ++c) child_add(c == 0 ? stp.y : stp.z, dv, c == c_lo, true);
        if (split && c_lo == 1) {
#pragma unroll
          for (int i = 0; i < kSQ; ++i) xr[i * kWave + lane] = dv[i];
        } else if (!split) {
          store_row(rdp, stp.x & 0xFFFF, dv);
          slot_put((stp.x >> 16) & 0xFF, dv);
        }
      }
      if (split) {
        site_barrier();
        if (wv < nit && (wv & 1) == 0) {
          const float* px = scr + (size_t)(wv + 1) * 2 * kSlotF;
#pragma unroll
          for (int i = 0; i < kSQ; ++i) dv[i] = dv[i] + px[i * kWave + lane];
          store_row(rdp, stp.x & 0xFFFF, dv);
          slot_put((stp.x >> 16) & 0xFF, dv);
        }
      }
      site_barrier();
      SITE_STAMP(2 + (s < 5 ? s : 5));
    }
  }

  // ---- root (the last stage's only task, wave 0): score + cotangent
  // (sankoff.py:187); its D and then its cotangent in its slot ----
  root_slot = (load_step(steps, pword(4 + S - 1)).x >> 16) & 0xFF;
  if (wv == 0) {
    float droot[kSQ], groot[kSQ];
    if constexpr (FWD)
      slot_get(root_slot, droot);
    else
      load_row(ni - 1, droot);
    float mn = droot[0];
#pragma unroll
    for (int i = 1; i < kSQ; ++i) mn = i < Q ? fminf(mn, droot[i]) : mn;
    float score;
    if (A.hard_root) {
      float cnt = 0.0f;
#pragma unroll
      for (int i = 0; i < kSQ; ++i) cnt += (i < Q && droot[i] == mn) ? 1.0f : 0.0f;
      const float r = 1.0f / cnt;
#pragma unroll
      for (int i = 0; i < kSQ; ++i) groot[i] = (i < Q && droot[i] == mn) ? r : 0.0f;
      score = mn;
    } else {
      // the minima (exactly 1 each) are summed apart and added last
      float ls = 0.0f, lt = 0.0f;
#pragma unroll
      for (int i = 0; i < kSQ; ++i) {
        groot[i] = i < Q ? fast_exp2((mn - droot[i]) * a) : 0.0f;
        const bool tie = i < Q && droot[i] == mn;
        ls += tie ? 0.0f : groot[i];
        lt += tie ? 1.0f : 0.0f;
      }
      const float sum = lt + ls;
      const float rs = __builtin_amdgcn_rcpf(sum);
#pragma unroll
      for (int i = 0; i < kSQ; ++i) groot[i] *= rs;
      score = fmaf(-bcoef, fast_log2(sum), mn);
    }
    if constexpr (FWD) {
      if (active && A.site_score) A.site_score[(size_t)tree * L + site] = score;
      const double tot = wave_sum_lane0(active ? (double)score : 0.0);
      if (lane == 0) A.part_tree[blockIdx.x] = tot;
    }
    const float f = active ? (A.dts ? as_const(A.dts)[tree] : 1.0f) : 0.0f;
#pragma unroll
    for (int i = 0; i < kSQ; ++i) groot[i] *= f;
    if constexpr (BWD) slot_put(root_slot, groot);
  }

  if constexpr (BWD) {
    // the forward's DP stores must be in L2 before the adjoint re-reads them
    // (other waves' rows; the loads below bypass nothing else)
    SITE_STAMP(8);
    if constexpr (FWD) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    SITE_STAMP(9);
    // dC accumulators: acc1 = sum r u^T (x K at the end), acc2 = sum of leaf
    // one-hot terms g e_code^T; 32 x 32 f32 blocks (rows = parent state i)
    f16v acc1, acc2;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc1[r] = 0.0f;
      acc2[r] = 0.0f;
    }
    const int mrow = lane & 31, khalf = lane >> 5;
    const int rrow = mrow < kSQ ? mrow : 0;  // rows >= 20: any finite data (discarded)
    // acc1 += r u^T over the wave's 64 sites (MFMA k = 2 sites)
    // acc1 += (scratch r)(scratch u)^T, the scratch already written
    auto outer_mfma = [&]() {
#ifdef SITE_DIAG_NOMFMA  // diagnostic: no dC outer products (wrong dC)
      wave_sync();
      return;
#endif
#if SITE_DC_BF16
      // r and u split exactly into three truncated 8-bit pieces each (hi + mid
      // + lo); the six products down to 2^-16 of |r u| (hl, lh, mm, mh, hm, hh,
      // smallest first) on v_mfma_f32_32x32x16_bf16, k = 16 sites: dropped
      // terms < 2^-23 |r u| per product (r, u >= 0: no cancellation), 24 MFMAs
      // of 32 cycles per 64 sites instead of 32 f32 MFMAs of 64
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int sg = 16 * t + 8 * khalf;  // this lane's 8 sites of the k-step
        u32x4 ah, am, al, bh, bm, bl;
        split3(xr + swz(rrow, sg), xr + swz(rrow, sg + 4), ah, am, al);
        split3(xu + swz(rrow, sg), xu + swz(rrow, sg + 4), bh, bm, bl);
        acc1 = mfma_bf(ah, bl, acc1);
        acc1 = mfma_bf(al, bh, acc1);
        acc1 = mfma_bf(am, bm, acc1);
        acc1 = mfma_bf(am, bh, acc1);
        acc1 = mfma_bf(ah, bm, acc1);
        acc1 = mfma_bf(ah, bh, acc1);
      }
#else
#pragma unroll
      for (int t4 = 0; t4 < 8; ++t4) {
        const int sg = khalf * 32 + 4 * t4;
        const float4 ra = *reinterpret_cast<const float4*>(xr + swz(rrow, sg));
        const float4 ub = *reinterpret_cast<const float4*>(xu + swz(rrow, sg));
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(ra.x, ub.x, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(ra.y, ub.y, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(ra.z, ub.z, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(ra.w, ub.w, acc1, 0, 0, 0);
      }
#endif
      wave_sync();
    };
    auto outer = [&](const float (&r)[kSQ], const float (&u)[kSQ]) {
#pragma unroll
      for (int i = 0; i < kSQ; ++i) {
        xr[swz(i, lane)] = r[i];
        xu[swz(i, lane)] = u[i];
      }
      wave_sync();
      outer_mfma();
    };
    // acc2 += g (sum of the leaf children's one-hot rows)^T on the bf16 matrix
    // core: g split exactly into three 8-bit pieces (hi + mid + lo, truncated,
    // residual < 2^-23 |g|) against exact 0 / 1 / 2 one-hot counts, k = 16
    // sites per v_mfma_f32_32x32x16_bf16 (12 per 64 sites instead of 32
    // 32x32x2 f32 MFMAs)
    auto leaf_hist = [&](const float (&g)[kSQ], int d0, int d1) {
#ifdef SITE_DIAG_NOMFMA
      return;
#endif
#pragma unroll
      for (int i = 0; i < kSQ; ++i) xr[swz(i, lane)] = g[i];
      wave_sync();
      const bool l0 = ((d0 >> 24) & 3) == kKindLeaf, l1 = ((d1 >> 24) & 3) == kKindLeaf;
      const uint32_t* c0 = reinterpret_cast<const uint32_t*>(lleaf + (d0 & 0xFFFF) * kWave);
      const uint32_t* c1 = reinterpret_cast<const uint32_t*>(lleaf + (d1 & 0xFFFF) * kWave);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int sg = 16 * t + 8 * khalf;  // this lane's 8 sites of the k-step
        u32x4 ph, pm, pl, pb;
        split3(xr + swz(rrow, sg), xr + swz(rrow, sg + 4), ph, pm, pl);
        const uint32_t w0[2] = {l0 ? c0[sg >> 2] : 0xFFFFFFFFu, l0 ? c0[(sg >> 2) + 1] : 0xFFFFFFFFu};
        const uint32_t w1[2] = {l1 ? c1[sg >> 2] : 0xFFFFFFFFu, l1 ? c1[(sg >> 2) + 1] : 0xFFFFFFFFu};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t bb[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int si = 2 * q + e;
            const uint32_t a0 = (w0[si >> 2] >> (8 * (si & 3))) & 0xFF, a1 = (w1[si >> 2] >> (8 * (si & 3))) & 0xFF;
            const int cnt = (a0 == (uint32_t)mrow ? 1 : 0) + (a1 == (uint32_t)mrow ? 1 : 0);
            bb[e] = cnt == 0 ? 0u : cnt == 1 ? 0x3F80u : 0x4000u;  // bf16 0, 1, 2
          }
          pb[q] = bb[0] | (bb[1] << 16);
        }
        const bf16x8 B = __builtin_bit_cast(bf16x8, pb);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ph), B, acc2, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, pm), B, acc2, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, pl), B, acc2, 0, 0, 0);
      }
      wave_sync();
    };
    // adjoint of one internal child with D = d under parent cotangent g:
    // w_ij = K_ij u_j / s_i, r_i = g_i / s_i; dC += r u^T (x K); gc_j = u_j sum_i K_ij r_i
    auto child_adj_rest = [&](const float (&u)[kSQ], float (&r)[kSQ], const float (&g)[kSQ],
                              float (&gc)[kSQ]) {
#pragma unroll
      for (int i = 0; i < kSQ; ++i) r[i] = i < Q ? g[i] * __builtin_amdgcn_rcpf(r[i]) : 0.0f;
#pragma unroll
      for (int i = 0; i < kSQ; ++i) {
        xr[swz(i, lane)] = r[i];
        xu[swz(i, lane)] = u[i];
      }
      wave_sync();
      // t_j = sum_i K_ij r_i: row i of K by scalar loads, r_i from the scratch
      f2 t2[kSQ / 2];
#pragma unroll
      for (int j = 0; j < kSQ / 2; ++j) t2[j] = pk(0.0f, 0.0f);
#pragma unroll 2
      for (int i = 0; i < Q; ++i) {
#ifdef SITE_DIAG_NOSMEM
        const cptr<float> kr = K;
#else
        const cptr<float> kr = K + i * kSQ;
#endif
        const float ri = xr[swz(i, lane)];
#pragma unroll
        for (int j = 0; j < kSQ; j += 2)
          t2[j / 2] = __builtin_elementwise_fma(pk(kr[j], kr[j + 1]), pk(ri, ri), t2[j / 2]);
      }
#pragma unroll
      for (int j = 0; j < kSQ; j += 2) {
        gc[j] = u[j] * t2[j / 2].x;
        gc[j + 1] = u[j + 1] * t2[j / 2].y;
      }
      outer_mfma();
    };
    auto child_adj = [&](const float (&d)[kSQ], const float (&g)[kSQ], float (&gc)[kSQ]) {
      float md, u[kSQ], r[kSQ];
      weights(d, md, u, r);
      child_adj_rest(u, r, g, gc);
    };
    // a cherry child: its row sums s from TS (the forward's mat-vec, bitwise)
    auto cherry_adj = [&](const I4& e, const float (&d)[kSQ], const float (&g)[kSQ],
                          float (&gc)[kSQ]) {
      if constexpr (!CH) {
        child_adj(d, g, gc);
        return;
      }
      float md, u[kSQ], r[kSQ];
      load_tab(tsg, pair_of(e), r);
      weights_u(d, md, u);
      child_adj_rest(u, r, g, gc);
    };
    // a 1e5-row child: u = 1 on every state, r_i = g_i / sum_j K_ij
    auto sent_adj = [&](const float (&g)[kSQ]) {
      float r[kSQ], u[kSQ];
#pragma unroll
      for (int i = 0; i < kSQ; ++i) {
        r[i] = g[i] * sinv[i];
        u[i] = i < Q ? 1.0f : 0.0f;
      }
      outer(r, u);
    };
    const bool want_marg = A.marg != nullptr;
    const rsrc_t rmg = make_rsrc(want_marg ? A.marg + (size_t)tree * ni * L * Q : A.dp, treebytes);
    int8_t* at = A.anc ? A.anc + (size_t)tree * ni * L + site : nullptr;
#ifndef SITE_EMIT_T
#define SITE_EMIT_T 0  // 1: marginal rows through the transposed store (slower, PERFLOG)
#endif
    auto emit = [&](int row, const float (&g)[kSQ]) {
      if (want_marg) {
        if (SITE_EMIT_T)
          store_row(rmg, row, g);
        else
          store_row_direct(rmg, row, g);
      }
      if (at && active) {
        float bv = g[0];
        int bi = 0;
#pragma unroll
        for (int i = 1; i < kSQ; ++i)
          if (i < Q && g[i] > bv) {
            bv = g[i];
            bi = i;
          }
        at[(size_t)row * L] = (int8_t)bi;
      }
    };
    // leaf / 1e5 children of a row with cotangent g
    auto leafish_adj = [&](const float (&g)[kSQ], int d0, int d1) {
      const int k0 = (d0 >> 24) & 3, k1 = (d1 >> 24) & 3;
      if (k0 == kKindLeaf || k1 == kKindLeaf) {
        leaf_hist(g, d0, d1);
        // a missing / out-of-range leaf state (code Q: trex's dropped scatter
        // leaves the all-1e5 row, sankoff.py:152) sends the T[Q] message,
        // which depends on C through log sum_j K_ij: its adjoint is the 1e5
        // row's (r_i = g_i / sum_j K_ij, u = 1), per lane, times the number
        // of such leaf children.  The histogram's column Q is discarded.
        const int nmiss = (k0 == kKindLeaf && leaf_code(d0) == Q ? 1 : 0) +
                          (k1 == kKindLeaf && leaf_code(d1) == Q ? 1 : 0);
        if (__any(active && nmiss != 0)) {
          const float fm = active ? (float)nmiss : 0.0f;
          float r[kSQ], u[kSQ];
#pragma unroll
          for (int i = 0; i < kSQ; ++i) {
            r[i] = fm * (g[i] * sinv[i]);
            u[i] = i < Q ? 1.0f : 0.0f;
          }
          outer(r, u);
        }
      }
      if (k0 == 0) sent_adj(g);
      if (k1 == 0) sent_adj(g);
    };
    // a row with cotangent g whose children are leaves / 1e5 rows / inline rows
    auto inline_adj = [&](int idx, const float (&g)[kSQ]) {
      const I4 e = load_step(inl, idx);
      emit(e.x, g);
      if (e.w > 1) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int desc = c == 0 ? e.y : e.z;
          if (((desc >> 24) & 3) == kKindInline) {
            const I4 e2 = load_step(inl, desc & 0xFFFF);
            float dc[kSQ], gc[kSQ];
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

    // children c in [c_lo, c_hi) of task row stp
    auto adj_task = [&](const I4& stp, int c_lo, int c_hi) {
        const int vslot = (stp.x >> 16) & 0xFF;
        int lf0 = 0x7F000000, lf1 = 0x7F000000;  // leaf / 1e5 children (kind 3 marks none)
        // one child at a time: its D row (task rows, height-2 inline rows:
        // re-read from HBM; height-1 rows: from the leaves), the parent's
        // cotangent re-read from its slot (fewer registers held across the
        // child's subtree)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          if (c < c_lo || c >= c_hi) continue;
          const int desc = c == 0 ? stp.y : stp.z;
          const int kind = (desc >> 24) & 3;
          if (kind == kKindInt || kind == kKindInline) {
            const I4 ie = kind == kKindInline ? load_step(inl, desc & 0xFFFF) : I4{desc & 0xFFFF, 0, 0, 2};
            float d[kSQ], g[kSQ], gc[kSQ];
            if (ie.w > 1 && keep_s) {
              // the forward's D and s rows of this child (no mat-vec)
              float sv[kSQ], md, u[kSQ];
              load_row(SITE_ADJ_ROW(ie.x), d);
              weights_u(d, md, u);
              load_row_r(rsr, SITE_ADJ_ROW(ie.x), sv);
              // lanes past L read 0 (their g is 0): keep r = g / s finite
#pragma unroll
              for (int i = 0; i < kSQ; ++i) sv[i] = active ? sv[i] : 1.0f;
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
            float g[kSQ];
            slot_get(vslot, g);
            emit(stp.x & 0xFFFF, g);
          } else {
            lf1 = desc;
          }
        }
        if (lf0 != 0x7F000000 || lf1 != 0x7F000000) {
          float g[kSQ];
          slot_get(vslot, g);
          leafish_adj(g, lf0, lf1);
        }
    };
    for (int s = S - 1; s >= 0; --s) {
      const int lo = pword(4 + s), hi = pword(5 + s);
      // a stage of at most kSWv / 2 tasks: one child per wave (the two
      // children's adjoints are independent: distinct slots, per-wave dC
      // accumulators; the c = 0 item emits the parent row)
      const bool split = 2 * (hi - lo) <= kSWv;
      const int nit = split ? 2 * (hi - lo) : hi - lo;
      for (int it = wv; it < nit; it += kSWv) {
        const int c_lo = split ? (it & 1) : 0;
        adj_task(load_step(steps, lo + (split ? it >> 1 : it)), c_lo, split ? c_lo + 1 : 2);
      }
      site_barrier();
      SITE_STAMP(10 + (S - 1 - s < 5 ? S - 1 - s : 5));
    }

    // ---- dC partial of the item: dC_ij = K_ij acc1_ij + acc2_ij per wave,
    // the waves summed in order through LDS (the slots / scratch are dead) ----
    double* red = reinterpret_cast<double*>(scr);  // [kSWv][Q][Q]
    const int Q2 = Q * Q;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = (r >> 2) * 8 + khalf * 4 + (r & 3), j = mrow;
      if (i < Q && j < Q)
        red[(size_t)wv * Q2 + i * Q + j] = (double)acc1[r] * (double)K[i * kSQ + j] + (double)acc2[r];
    }
    __syncthreads();
    const int nb = A.B * A.tiles;
    for (int e = threadIdx.x; e < Q2; e += kSWv * kWave) {
      double tsum = red[e];
#pragma unroll
      for (int w = 1; w < kSWv; ++w) tsum += red[(size_t)w * Q2 + e];
      A.part_dc[(size_t)e * nb + blockIdx.x] = tsum;
    }
    SITE_STAMP(16);
  }
}

}  // namespace

#ifdef TREX_SITE_TIMING
extern "C" int trex_debug_site_times(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_site_t), sizeof(g_site_t)) == hipSuccess ? 0 : -4;
}
#endif

int site_tiles(int L) { return (L + kWave - 1) / kWave; }

size_t site_lds_bytes(int n_slots, int nl, int ni) {
  const size_t b = ((size_t)n_slots * kSlotF + (size_t)kSWv * 2 * kSlotF + kTabF + lp_tree_ints(ni)) * 4 +
                   (size_t)nl * kWave;
  return (b + 15) & ~(size_t)15;
}

// host-side eligibility (the cost-dependent mode is decided on the device):
// soft, 4 < Q <= 20, every tree has a lane program whose slots fit the LDS
bool site_srow_on() {
  const char* e = std::getenv("TREX_SITE_SROW");  // "0": the adjoint recomputes s (A/B)
  return !(e && e[0] == '0');
}

bool site_eligible(const WideCall& c, int lp_slots) {
  if (!c.soft || c.Q <= 4 || c.Q > kSQ || lp_slots < 0) return false;
  const char* e = std::getenv("TREX_SITE");  // "0": the state-parallel kernel (A/B)
  if (e && e[0] == '0') return false;
  if ((int64_t)c.ni * c.L * c.Q * 4 > 0x7FFFFFF0LL) return false;
  return site_lds_bytes(lp_slots, c.nl, c.ni) <= 160 * 1024;
}

int site_run(const char* fn, const WideCall& c, const int32_t* lanes, int lp_slots,
             const int* flag, const float* kg) {
  const int tiles = site_tiles(c.L);
  const size_t lds = site_lds_bytes(lp_slots, c.nl, c.ni);
  if ((int64_t)c.B * tiles > 0x7FFFFFFF) return set_error(TREX_E_ARG, "%s: grid too large", fn);
  hipStream_t st = (hipStream_t)c.stream;
  SiteArgs A;
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
  {
    const char* e = std::getenv("TREX_SITE_CHERRY");  // read per call (tests flip it)
    A.cherry = !(e && e[0] == '0');
  }
  A.flag = flag;
  A.n_slots = lp_slots;
  auto go = [&](auto kernel) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kernel, dim3((int)nb), dim3(kSWv * kWave), lds, st, A);
  };
  const bool ks = A.srow != nullptr;
  if (c.Q == kSQ && !A.cherry) {  // A/B: no cherry tables, no kept s rows
    if (c.phase == 1)
      go(sankoff_site_kernel<1, kSQ, false, false>);
    else if (c.phase == 2)
      go(sankoff_site_kernel<2, kSQ, false, false>);
    else
      go(sankoff_site_kernel<3, kSQ, false, false>);
  } else if (c.Q == kSQ) {
    if (c.phase == 1)
      go(sankoff_site_kernel<1, kSQ>);
    else if (c.phase == 2)
      go(sankoff_site_kernel<2, kSQ>);
    else if (ks)
      go(sankoff_site_kernel<3, kSQ, true>);
    else
      go(sankoff_site_kernel<3, kSQ>);
  } else {
    if (c.phase == 1)
      go(sankoff_site_kernel<1, 0>);
    else if (c.phase == 2)
      go(sankoff_site_kernel<2, 0>);
    else if (ks)
      go(sankoff_site_kernel<3, 0, true>);
    else
      go(sankoff_site_kernel<3, 0>);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

}  // namespace trex
