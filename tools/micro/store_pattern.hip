// Store-pattern microbenchmark: achievable HBM write bandwidth of the Sankoff
// DP-table write pattern vs. streaming (tuning aid, not part of the library).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

// one wave per block; block = (tree, tile); per step writes Q rows of 64*W floats
template <int W>
__global__ __launch_bounds__(64) void rows_kernel(float* dp, int B, int tiles, int n_int, int Q, int L, int grouped) {
  int b = blockIdx.x;
  const int nb = B * tiles;
  if (grouped) { const int per = (nb + 7) / 8; b = (b & 7) * per + (b >> 3); if (b >= nb) return; }
  const int tree = b / tiles, tile = b % tiles;
  const int site = (tile * 64 + threadIdx.x) * W;
  if (site >= L) return;
  float* base = dp + (size_t)tree * n_int * Q * L + site;
  float v = (float)threadIdx.x;
  for (int k = 0; k < n_int; ++k) {
    for (int q = 0; q < Q; ++q) {
      float* p = base + ((size_t)k * Q + q) * L;
      if constexpr (W == 4) *reinterpret_cast<float4*>(p) = make_float4(v, v, v, v);
      else if constexpr (W == 2) *reinterpret_cast<float2*>(p) = make_float2(v, v);
      else *p = v;
    }
    v += 1.0f;
  }
}

// tile-major layout [B][n_int][tiles][Q][64*W]: a wave's Q rows are contiguous
template <int W>
__global__ __launch_bounds__(64) void tilemajor_kernel(float* dp, int B, int tiles, int n_int, int Q, int grouped) {
  int b = blockIdx.x;
  const int nb = B * tiles;
  if (grouped) { const int per = (nb + 7) / 8; b = (b & 7) * per + (b >> 3); if (b >= nb) return; }
  const int tree = b / tiles, tile = b % tiles;
  float v = (float)threadIdx.x;
  const size_t chunk = (size_t)Q * 64 * W;
  for (int k = 0; k < n_int; ++k) {
    float* p = dp + (((size_t)tree * n_int + k) * tiles + tile) * chunk + threadIdx.x * W;
    for (int q = 0; q < Q; ++q) {
      if constexpr (W == 4) *reinterpret_cast<float4*>(p + q * 64 * W) = make_float4(v, v, v, v);
      else *reinterpret_cast<float*>(p + q * 64 * W) = v;
    }
    v += 1.0f;
  }
}

// site-major layout [B][n_int][L][Q]: a lane's Q=4 states are one dwordx4
// store, a wave writes 1 KiB contiguous per node
__global__ __launch_bounds__(64) void sitemajor_kernel(float* dp, int B, int tiles, int n_int, int L, int grouped) {
  int b = blockIdx.x;
  const int nb = B * tiles;
  if (grouped) { const int per = (nb + 7) / 8; b = (b & 7) * per + (b >> 3); if (b >= nb) return; }
  const int tree = b / tiles, tile = b % tiles;
  const int site = tile * 64 + threadIdx.x;
  if (site >= L) return;
  float v = (float)threadIdx.x;
  float4* base = reinterpret_cast<float4*>(dp) + (size_t)tree * n_int * L + site;
  for (int k = 0; k < n_int; ++k) {
    base[(size_t)k * L] = make_float4(v, v, v, v);
    v += 1.0f;
  }
}

__global__ void stream_kernel(float4* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_float4(1, 2, 3, 4);
}

int main() {
  const int B = 128, n_int = 31, Q = 4, L = 5000;
  const size_t n = (size_t)B * n_int * Q * L;
  const int tiles64 = (L + 63) / 64;
  float* dp;
  hipMalloc(&dp, (n + 64 * 64) * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double s = ms / 20 * 1e-3;
    printf("%-40s %8.1f us  %7.1f GB/s\n", name, s * 1e6, n * 4 / s / 1e9);
  };
  for (int g = 0; g < 2; ++g) {
    char nm[64];
    snprintf(nm, 64, "rows W=1 grouped=%d", g);
    timeit(nm, [&] { int nb = B * tiles64; hipLaunchKernelGGL(rows_kernel<1>, dim3((nb + 7) / 8 * 8), dim3(64), 0, 0, dp, B, tiles64, n_int, Q, L, g); });
    snprintf(nm, 64, "rows W=2 grouped=%d", g);
    int t2 = (L + 127) / 128;
    timeit(nm, [&] { int nb = B * t2; hipLaunchKernelGGL(rows_kernel<2>, dim3((nb + 7) / 8 * 8), dim3(64), 0, 0, dp, B, t2, n_int, Q, L, g); });
    snprintf(nm, 64, "rows W=4 grouped=%d", g);
    int t4 = (L + 255) / 256;
    timeit(nm, [&] { int nb = B * t4; hipLaunchKernelGGL(rows_kernel<4>, dim3((nb + 7) / 8 * 8), dim3(64), 0, 0, dp, B, t4, n_int, Q, L, g); });
    snprintf(nm, 64, "tilemajor W=1 grouped=%d", g);
    timeit(nm, [&] { int nb = B * 78; hipLaunchKernelGGL(tilemajor_kernel<1>, dim3((nb + 7) / 8 * 8), dim3(64), 0, 0, dp, B, 78, n_int, Q, g); });
    snprintf(nm, 64, "tilemajor W=4 grouped=%d", g);
    timeit(nm, [&] { int nb = B * 19; hipLaunchKernelGGL(tilemajor_kernel<4>, dim3((nb + 7) / 8 * 8), dim3(64), 0, 0, dp, B, 19, n_int, Q, g); });
  }
  for (int g = 0; g < 2; ++g) {
    char nm[64];
    snprintf(nm, 64, "sitemajor x4 grouped=%d", g);
    timeit(nm, [&] { int nb = B * tiles64; hipLaunchKernelGGL(sitemajor_kernel, dim3((nb + 7) / 8 * 8), dim3(64), 0, 0, dp, B, tiles64, n_int, L, g); });
  }
  timeit("stream float4", [&] { hipLaunchKernelGGL(stream_kernel, dim3(8192), dim3(256), 0, 0, (float4*)dp, n / 4); });
  return 0;
}
