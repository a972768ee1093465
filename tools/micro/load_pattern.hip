// FETCH_SIZE calibration on gfx950 (tuning aid): known byte counts read with
// the Sankoff adjoint's access pattern (4 B/lane buffer loads of 256-B DP-row
// chunks, 4 rows per step) and with 16 B/lane streaming loads.  Run under
// rocprofv3 --pmc FETCH_SIZE; the ratio FETCH_SIZE*1024 / bytes is the
// correction factor for that access width.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void rows_load(const float* dp, float* out, int B, int tiles,
                                                int n_int, int Q, int L) {
  const int per = (B * tiles + 7) / 8;
  const int b = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (b >= B * tiles) return;
  const int tree = b / tiles, tile = b % tiles;
  const int site = tile * 64 + threadIdx.x;
  if (site >= L) return;
  const float* base = dp + (size_t)tree * n_int * Q * L + site;
  float acc = 0.f;
  for (int k = n_int - 1; k >= 0; --k)
    for (int q = 0; q < Q; ++q) acc += base[((size_t)k * Q + q) * L];
  if (acc == 123.456f) out[0] = acc;
}

__global__ void stream_load(const float4* p, size_t n, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = p[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 123.456f) out[0] = acc;
}

int main() {
  const int B = 128, n_int = 31, Q = 4, L = 5000, tiles = (L + 63) / 64;
  const size_t n = (size_t)B * n_int * Q * L;
  float *dp, *out;
  if (hipMalloc(&dp, n * 4) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(dp, 0, n * 4);
  for (int i = 0; i < 3; ++i) {
    hipLaunchKernelGGL(rows_load, dim3((B * tiles + 7) / 8 * 8), dim3(64), 0, 0, dp, out, B, tiles, n_int, Q, L);
    hipLaunchKernelGGL(stream_load, dim3(8192), dim3(256), 0, 0, (const float4*)dp, n / 4, out);
  }
  (void)hipDeviceSynchronize();
  printf("bytes per launch: %zu\n", n * 4);
  return 0;
}
