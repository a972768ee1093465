// Memory-pattern microbenchmark for the fused Sankoff fwd + adjoint (tuning
// aid, not part of the library): each wave writes its tree's n_int DP rows
// (forward) and reads them back in reverse order (adjoint), with no
// arithmetic, in the two candidate HBM layouts:
//   rows      [B][n_int][Q][L]  4 B per lane per row, Q rows per node
//   sitemajor [B][n_int][L][Q]  one 16-B (dwordx4) access per lane per node
// plus the write-only and read-only halves.  C4 shard shape.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int Q = 4;

template <bool SITEMAJOR, bool WR, bool RD>
__global__ __launch_bounds__(64) void pattern(float* dp, float* out, int B, int tiles, int n_int, int L) {
  const int nb = B * tiles;
  const int per = (nb + 7) / 8;
  const int b = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (b >= nb) return;
  const int tree = b / tiles, tile = b % tiles;
  const int site = tile * 64 + threadIdx.x;
  if (site >= L) return;
  float v = (float)threadIdx.x;
  if constexpr (WR) {
    for (int k = 0; k < n_int; ++k) {
      if constexpr (SITEMAJOR) {
        reinterpret_cast<float4*>(dp)[((size_t)tree * n_int + k) * L + site] = make_float4(v, v + 1, v + 2, v + 3);
      } else {
        float* p = dp + ((size_t)tree * n_int + k) * Q * L + site;
        for (int q = 0; q < Q; ++q) p[(size_t)q * L] = v + q;
      }
      v += 1.0f;
    }
  }
  if constexpr (RD) {
    float acc = 0.f;
    for (int k = n_int - 1; k >= 0; --k) {
      if constexpr (SITEMAJOR) {
        const float4 x = reinterpret_cast<const float4*>(dp)[((size_t)tree * n_int + k) * L + site];
        acc += x.x + x.y + x.z + x.w;
      } else {
        const float* p = dp + ((size_t)tree * n_int + k) * Q * L + site;
        for (int q = 0; q < Q; ++q) acc += p[(size_t)q * L];
      }
    }
    if (acc == 123.456f) out[0] = acc;
  }
}

int main() {
  const int B = 128, n_int = 31, L = 5000, tiles = (L + 63) / 64;
  const size_t n = (size_t)B * n_int * Q * L;
  float *dp, *out;
  if (hipMalloc(&dp, n * 4) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(dp, 0, n * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = (B * tiles + 7) / 8 * 8;
  auto timeit = [&](const char* name, auto kern, double passes) {
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, dp, out, B, tiles, n_int, L);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, dp, out, B, tiles, n_int, L);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double s = ms / 20 * 1e-3;
    printf("%-28s %8.1f us  %7.1f GB/s\n", name, s * 1e6, passes * n * 4 / s / 1e9);
  };
  timeit("rows write", pattern<false, true, false>, 1);
  timeit("rows read", pattern<false, false, true>, 1);
  timeit("rows write+read", pattern<false, true, true>, 2);
  timeit("sitemajor write", pattern<true, true, false>, 1);
  timeit("sitemajor read", pattern<true, false, true>, 1);
  timeit("sitemajor write+read", pattern<true, true, true>, 2);
  return 0;
}
