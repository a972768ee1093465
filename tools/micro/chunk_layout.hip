// Read-rate micro-benchmark for the C5 Gram's operand stream: an N x K f32
// matrix (N = 511, K = 200 000: C5's S, 409 MB) read in K chunks of 16
// columns, all N rows per chunk, one 512-thread workgroup per CU walking a
// contiguous K range -- (a) row-major [N][K]: a chunk is N segments of 64 B,
// rows 800 KB apart; (b) chunk-major [K/16][N][16]: a chunk is one
// contiguous 32 KB block.  Same loads in flight in both (D chunks ahead).
//   hipcc --offload-arch=gfx950 -O3 -o chunk_layout chunk_layout.hip && ./chunk_layout
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int N = 511, K = 200000, CK = 16, NT = 512;
constexpr int F4 = N * CK / 4;             // float4 per chunk (2044)
constexpr int PER = (F4 + NT - 1) / NT;    // float4 per thread per chunk (4)

template <bool CHUNK_MAJOR, int D>
__global__ __launch_bounds__(NT) void reader(const float4* __restrict__ x, int chunks_per_wg, float* out) {
  const int nck = K / CK;
  const int c0 = blockIdx.x * chunks_per_wg;
  const int c1 = min(nck, c0 + chunks_per_wg);
  float acc = 0.0f;
  float4 buf[D][PER];
  auto issue = [&](int c, float4 (&b)[PER]) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int e = threadIdx.x + NT * p;  // float4 index inside the chunk
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < F4 && c < c1) {
        size_t idx;
        if (CHUNK_MAJOR) {
          idx = (size_t)c * F4 + e;
        } else {
          const int row = e / (CK / 4), q = e % (CK / 4);
          idx = ((size_t)row * K + (size_t)c * CK) / 4 + q;
        }
        v = x[idx];
      }
      b[p] = v;
    }
  };
#pragma unroll
  for (int d = 0; d < D; ++d) issue(c0 + d, buf[d]);
  for (int c = c0; c < c1; c += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int p = 0; p < PER; ++p) acc += buf[d][p].x + buf[d][p].y + buf[d][p].z + buf[d][p].w;
      issue(c + d + D, buf[d]);
    }
  }
  if (acc == 1234.5f) out[0] = acc;  // keeps the loads
}

template <bool CM, int D>
float run(const float4* x, float* out, int wgs) {
  const int nck = K / CK;
  const int per = (nck + wgs - 1) / wgs;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) reader<CM, D><<<wgs, NT>>>(x, per, out);
  hipEventRecord(e0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) reader<CM, D><<<wgs, NT>>>(x, per, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps * 1e3f;  // us
}

int main() {
  const size_t bytes = (size_t)N * K * 4;
  float4* x;
  float* out;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  hipMemset(x, 0, bytes);
  const int wgs = 256;
  printf("N %d K %d: %.1f MB, %d workgroups of %d threads\n", N, K, bytes / 1e6, wgs, NT);
  for (int rep = 0; rep < 2; ++rep) {
    float a1 = run<false, 1>(x, out, wgs), b1 = run<true, 1>(x, out, wgs);
    float a2 = run<false, 2>(x, out, wgs), b2 = run<true, 2>(x, out, wgs);
    float a4 = run<false, 4>(x, out, wgs), b4 = run<true, 4>(x, out, wgs);
    printf("chunks in flight 1: row-major %.1f us (%.2f TB/s)  chunk-major %.1f us (%.2f TB/s)\n", a1,
           bytes / a1 / 1e6, b1, bytes / b1 / 1e6);
    printf("chunks in flight 2: row-major %.1f us (%.2f TB/s)  chunk-major %.1f us (%.2f TB/s)\n", a2,
           bytes / a2 / 1e6, b2, bytes / b2 / 1e6);
    printf("chunks in flight 4: row-major %.1f us (%.2f TB/s)  chunk-major %.1f us (%.2f TB/s)\n", a4,
           bytes / a4 / 1e6, b4, bytes / b4 / 1e6);
  }
  hipFree(x);
  hipFree(out);
  return 0;
}
