// libtrexhip.so -- synthetic data on the device:
// trex's ground-truth generator (src/trex/ground_truth.py:20-52 mutate,
// :112-197 generate_groundtruth) and iid uniform leaf states, so C4 / C5-size
// alignments are produced where they are consumed instead of on the host.
//
// Same process as the reference, different random numbers: trex draws with
// JAX's threefry PRNG (not available here); this file uses a counter-based
// generator, r(seed, stream, counter) = mix(seed ^ mix(stream << 32 | counter))
// with mix = the splitmix64 finaliser, so every draw is a pure function of
// its indices (no state, any launch shape, bitwise reproducible; restated in
// numpy in oracle/datagen_ref.py, which the tests match bit for bit).
//
//   mutate(parent -> child): exactly n_mutations distinct sites (Floyd's
//     sampling without replacement, draws on stream 2*child+1) get
//     (x + 1 + r % (Q - 1)) mod Q (stream 2*child, counter = site);
//   generate_groundtruth: a balanced tree, root (last row) all zero, parents
//     processed from the root down (parent n_all-1-i has children 2(p-nl)
//     and 2(p-nl)+1, ground_truth.py:165-178), one launch per tree level.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "trex_common.h"

namespace trex {

namespace {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ uint64_t draw(uint64_t seed, uint64_t stream, uint64_t counter) {
  return mix64(seed ^ mix64((stream << 32) | (counter & 0xFFFFFFFFull)));
}

constexpr int kMaxMut = 1024;  // sites per child held in LDS

// Floyd's algorithm: n_mut distinct sites of [0, L) per child (one thread
// per child; n_mut is small: trex uses 1-50 mutations per edge)
__global__ void choose_sites_kernel(uint64_t seed, int L, int n_mut, int child0, int nchild,
                                    int* __restrict__ sites) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nchild) return;
  const int child = child0 + t;
  int* s = sites + (size_t)t * n_mut;
  int k = 0;
  for (int j = L - n_mut; j < L; ++j) {
    const int r = (int)(draw(seed, 2ull * child + 1, (uint64_t)j) % (uint64_t)(j + 1));
    bool seen = false;
    for (int q = 0; q < k; ++q) seen |= s[q] == r;
    s[k++] = seen ? j : r;
  }
}

// one tree level: children [child0, child0 + nchild) from their parents
__global__ __launch_bounds__(256) void mutate_level_kernel(uint64_t seed, int nl, int L, int Q,
                                                           int n_mut, int child0,
                                                           const int* __restrict__ sites,
                                                           int8_t* __restrict__ seqs) {
  __shared__ int ms[kMaxMut];
  const int t = blockIdx.y;
  const int child = child0 + t;
  const int parent = nl + child / 2;  // children 2(p - nl), 2(p - nl) + 1
  for (int q = threadIdx.x; q < n_mut; q += blockDim.x) ms[q] = sites[(size_t)t * n_mut + q];
  __syncthreads();
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= L) return;
  bool hit = false;
  for (int q = 0; q < n_mut; ++q) hit |= ms[q] == s;
  int x = seqs[(size_t)parent * L + s];
  if (hit) x = (x + 1 + (int)(draw(seed, 2ull * child, (uint64_t)s) % (uint64_t)(Q - 1))) % Q;
  seqs[(size_t)child * L + s] = (int8_t)x;
}

__global__ __launch_bounds__(256) void uniform_states_kernel(uint64_t seed, int64_t n, int Q,
                                                             int8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int8_t)(draw(seed, (uint64_t)(i >> 32) + 0x100000000ull, (uint64_t)i) % (uint64_t)Q);
}

// ---- NK-model evolution along a tree (nk_model.py:116-278) ---------------
// One workgroup per node of a BFS level (its parent is finished): the
// parent's sequence in LDS, then branch_length Metropolis steps, each a
// coupled (one site + its K interactions) or independent (per-site
// Bernoulli(rate)) redraw, accepted with probability min(1, exp(f_new -
// f_cur)).  Fitness = mean over sites of fitness[i][sum_j s(site_j) Q^j]
// (site_0 = i, site_j = interactions[i][j - 1]), summed in 2^-40 fixed
// point (int64: order-free, bitwise reproducible).  Draws per BFS slot n
// (the reference's sorted_nodes index): stream 4n: rate noise (2
// uniforms), stream 4n + 1: step b's coupled decision / site / acceptance
// (counters 4b .. 4b + 2), stream 4n + 2: new states (counter b L + i),
// stream 4n + 3: independent-mutation mask.
__device__ __forceinline__ double unit53(uint64_t r) { return (double)(r >> 11) * 0x1.0p-53; }

// Gumbel(0, 1) noise for step `count` of a device loop -- the reference's
// fresh jax.random.gumbel(step_key) per step (tree.py:71,
// tests/test_convergence.py:258-261) as a pure function of (seed, step,
// index): u = (r >> 11 + 1/2) 2^-53 in (0, 1), g = -log(-log u) in double,
// rounded to f32 (restated in oracle/datagen_ref.py).  count: the device
// step state's first word (trex_step_advance), NULL = step 0.
__global__ __launch_bounds__(256) void gumbel_kernel(uint64_t seed, const int* __restrict__ count,
                                                     int64_t n, float* __restrict__ out) {
  const uint64_t step = count ? (uint64_t)(uint32_t)count[0] : 0ull;
  const uint64_t sk = mix64(seed ^ (0x6A09E667F3BCC909ull * (step + 1ull)));
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t r = draw(sk, 0x7FFF0000ull + (uint64_t)(i >> 32), (uint64_t)i);
    const double u = ((double)(r >> 11) + 0.5) * 0x1.0p-53;
    out[i] = (float)(-log(-log(u)));
  }
}
__device__ __forceinline__ float unit24(uint64_t r) { return (float)(r >> 40) * 0x1.0p-24f; }

__device__ __forceinline__ int64_t nk_fixed(float v) { return (int64_t)((double)v * 0x1.0p40); }

template <int BS>
__device__ __forceinline__ int64_t block_sum_i64(int64_t v, int64_t* red) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  int64_t t = 0;
  for (int i = 0; i < BS / 64; ++i) t += red[i];
  return t;
}

template <int BS>
__device__ int64_t nk_fitness_fixed(const int8_t* seq, int L, int Q, int K,
                                    const int* __restrict__ inter, const float* __restrict__ fit,
                                    int64_t tw, int64_t* red) {
  int64_t acc = 0;
  for (int i = threadIdx.x; i < L; i += BS) {
    int64_t idx = seq[i];
    int64_t pw = Q;
    for (int j = 0; j < K; ++j, pw *= Q) idx += (int64_t)seq[inter[(size_t)i * K + j]] * pw;
    acc += nk_fixed(fit[(size_t)i * tw + idx]);
  }
  return block_sum_i64<BS>(acc, red);
}

constexpr int kNkBlock = 256;

__global__ __launch_bounds__(kNkBlock) void nk_evolve_level_kernel(
    uint64_t seed, const int* __restrict__ order, int slot0, const int* __restrict__ parent, int L,
    int Q,
    int K, const int* __restrict__ inter, const float* __restrict__ fit, int64_t tw,
    float mutation_rate, float noise_std, float coupled_prob, int branch_length,
    int8_t* __restrict__ seqs) {
  extern __shared__ __attribute__((aligned(16))) int8_t nk_lds[];
  __shared__ int64_t red[kNkBlock / 64];
  int8_t* cur = nk_lds;
  int8_t* prop = nk_lds + L;
  const int slot = slot0 + (int)blockIdx.x;
  const int node = order[slot];
  const int par = parent[node];
  const uint64_t sb = 4ull * (uint64_t)slot;
  for (int i = threadIdx.x; i < L; i += kNkBlock) cur[i] = seqs[(size_t)par * L + i];
  __syncthreads();
  float rate = fminf(mutation_rate, 1.0f);
  if (noise_std != 0.0f) {  // rate * exp(N(0, 1) * std), Box-Muller
    const double u1 = 1.0 - unit53(draw(seed, sb, 0)), u2 = unit53(draw(seed, sb, 1));
    const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    rate = fminf((float)((double)mutation_rate * exp(z * (double)noise_std)), 1.0f);
  }
  int64_t fcur = nk_fitness_fixed<kNkBlock>(cur, L, Q, K, inter, fit, tw, red);
  for (int b = 0; b < branch_length; ++b) {
    const bool coupled = unit24(draw(seed, sb + 1, 4ull * b)) < coupled_prob;
    const int site0 = (int)(draw(seed, sb + 1, 4ull * b + 1) % (uint64_t)L);
    for (int i = threadIdx.x; i < L; i += kNkBlock) {
      bool m;
      if (coupled) {
        m = i == site0;
        for (int j = 0; j < K; ++j) m |= inter[(size_t)site0 * K + j] == i;
      } else {
        m = unit24(draw(seed, sb + 3, (uint64_t)b * L + i)) < rate;
      }
      const int v = (int)(draw(seed, sb + 2, (uint64_t)b * L + i) % (uint64_t)Q);
      prop[i] = m ? (int8_t)v : cur[i];
    }
    __syncthreads();
    const int64_t fprop = nk_fitness_fixed<kNkBlock>(prop, L, Q, K, inter, fit, tw, red);
    const double delta = (double)(fprop - fcur) * 0x1.0p-40 / (double)L;
    const bool accept = delta >= 0.0 || unit53(draw(seed, sb + 1, 4ull * b + 2)) < exp(delta);
    if (accept) {
      for (int i = threadIdx.x; i < L; i += kNkBlock) cur[i] = prop[i];
      fcur = fprop;
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < L; i += kNkBlock) seqs[(size_t)node * L + i] = cur[i];
}

}  // namespace

}  // namespace trex

using namespace trex;

extern "C" int64_t trex_datagen_workspace_bytes(int n_leaves, int n_mutations) {
  if (n_leaves <= 0 || n_mutations < 0) return 0;
  return (int64_t)n_leaves * (n_mutations > 0 ? n_mutations : 1) * 4 + 256;
}

extern "C" int trex_datagen_groundtruth(uint64_t seed, int n_leaves, int L, int Q, int n_mutations,
                                        int8_t* seqs, void* workspace, int64_t workspace_bytes,
                                        void* stream) {
  const char* fn = "trex_datagen_groundtruth";
  if (n_leaves < 2 || (n_leaves & (n_leaves - 1)) != 0)
    return set_error(TREX_E_ARG, "%s: n_leaves must be a power of 2 (got %d)", fn, n_leaves);
  if (L <= 0 || Q < 2 || Q > 127 || n_mutations < 0 || n_mutations > L || n_mutations > kMaxMut ||
      !seqs || !workspace)
    return set_error(TREX_E_ARG, "%s: bad arguments (L=%d Q=%d n_mutations=%d)", fn, L, Q,
                     n_mutations);
  if (workspace_bytes < trex_datagen_workspace_bytes(n_leaves, n_mutations))
    return set_error(TREX_E_ARG, "%s: workspace too small", fn);
  const int nl = n_leaves, n_all = 2 * nl - 1;
  hipStream_t st = (hipStream_t)stream;
  // the root (last row) is all zero (ground_truth.py:160)
  if (hipMemsetAsync(seqs + (size_t)(n_all - 1) * L, 0, (size_t)L, st) != hipSuccess)
    return set_error(TREX_E_HIP, "%s: memset failed", fn);
  int* sites = static_cast<int*>(workspace);
  // parents i = 0 .. n_anc-1 from the root down; depth d holds i in
  // [2^d - 1, 2^(d+1) - 1), whose children are a contiguous block of rows
  for (int lo = 0, width = 1; lo < nl - 1; lo += width, width *= 2) {
    const int hi = lo + width;                 // parents i in [lo, hi)
    const int p_lo = n_all - hi, p_hi = n_all - lo;  // parent rows [p_lo, p_hi)
    const int child0 = 2 * (p_lo - nl), nchild = 2 * (p_hi - p_lo);
    if (n_mutations > 0)
      hipLaunchKernelGGL(choose_sites_kernel, dim3((nchild + 63) / 64), dim3(64), 0, st, seed, L,
                         n_mutations, child0, nchild, sites);
    hipLaunchKernelGGL(mutate_level_kernel, dim3((L + 255) / 256, nchild), dim3(256), 0, st, seed,
                       nl, L, Q, n_mutations, child0, sites, seqs);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

extern "C" int trex_gumbel_noise(uint64_t seed, const void* state, int64_t n, float* out,
                                 void* stream) {
  if (n <= 0 || !out) return set_error(TREX_E_ARG, "trex_gumbel_noise: bad arguments");
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(gumbel_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     (hipStream_t)stream, seed, static_cast<const int*>(state), n, out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "trex_gumbel_noise: %s", hipGetErrorString(e));
  return TREX_OK;
}

extern "C" int trex_datagen_uniform_states(uint64_t seed, int64_t n, int Q, int8_t* out,
                                           void* stream) {
  if (n <= 0 || Q < 1 || Q > 127 || !out)
    return set_error(TREX_E_ARG, "trex_datagen_uniform_states: bad arguments");
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(uniform_states_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)),
                     dim3(256), 0, (hipStream_t)stream, seed, n, Q, out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_error(TREX_E_HIP, "trex_datagen_uniform_states: %s", hipGetErrorString(e));
  return TREX_OK;
}

extern "C" int trex_datagen_nk_tree(uint64_t seed, int n_nodes, int L, int Q, int K,
                                    const int* interactions, const float* fitness,
                                    const int* parent, const int* order, const int* level_offsets,
                                    int n_levels, float mutation_rate, float noise_std,
                                    float coupled_prob, int branch_length, int8_t* seqs,
                                    void* stream) {
  const char* fn = "trex_datagen_nk_tree";
  if (n_nodes < 1 || L < 1 || L > 65536 || Q < 2 || Q > 127 || K < 0 || K > 16 || !fitness ||
      (K > 0 && !interactions) || !parent || !order || !level_offsets || n_levels < 1 || !seqs ||
      branch_length < 0 || !finite_f32(mutation_rate) || !finite_f32(noise_std) ||
      !finite_f32(coupled_prob))
    return set_error(TREX_E_ARG, "%s: bad arguments", fn);
  double tw = 1.0;
  for (int j = 0; j <= K; ++j) tw *= Q;
  if (tw > 2147483647.0) return set_error(TREX_E_ARG, "%s: Q^(K+1) too large", fn);
  const int lds = 2 * L;
  if (lds > 65536 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(nk_evolve_level_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return set_error(TREX_E_HIP, "%s: LDS size", fn);
  hipStream_t st = (hipStream_t)stream;
  // level 0 is the root (copied in by the caller); host-side offsets; a
  // level's nodes are independent (their parents are done)
  for (int lv = 1; lv < n_levels; ++lv) {
    const int lo = level_offsets[lv], hi = level_offsets[lv + 1];
    if (hi <= lo) continue;
    hipLaunchKernelGGL(nk_evolve_level_kernel, dim3(hi - lo), dim3(kNkBlock), lds, st, seed,
                       order, lo, parent, L, Q, K, interactions, fitness, (int64_t)tw,
                       mutation_rate, noise_std, coupled_prob, branch_length, seqs);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}
