// Store-data register reuse on MI355X (gfx950): does a 128-bit buffer store
// still write its own bytes when the very next instruction overwrites its
// data VGPRs?  (Root cause of the round-5 corrupted DP-row bytes of the
// lane-per-site kernel: DESIGN.md section 5.8, tools/isa_store_guard.py.)
//
// Each wave stores ITERS rows of 64 x 16 B (one buffer_store_dwordx4 per
// row, the value a function of (wave, row, lane, dword)) and right behind
// every store runs one of these sequences on the data registers v[40:43]:
//   0 nop      s_nop 4, then a VALU write          (control: wait states)
//   1 valu     v_mov_b32 v40..v43 at once         (VALU write, SGPR soffset)
//   2 valu0    the same after a store whose soffset is the constant 0
//              (the case the ISA's wait-state table names)
//   3 ds       ds_read_b128 v[40:43] at once      (LDS return into the data)
//   4 vmem     buffer_load_dwordx4 v[40:43] at once (VMEM return into the data)
//   5 nop0     s_nop 0 (one wait state), then the VALU write
//   6 valu2    one unrelated VALU, then the VALU write (distance 2)
// The host counts the 16-byte rows whose bytes differ from the expected
// values.  Hand-placed registers: the sequences are inline asm, so the
// compiler's hazard recognizer does not insert anything between them.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/store_reuse tools/micro/store_reuse.hip
// run:   tools/micro/store_reuse [iters]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t expect(uint32_t wave, uint32_t row, uint32_t lane, uint32_t d) {
  return (wave * 2654435761u) ^ (row * 40503u) ^ (lane << 8) ^ d ^ 0x5A5A0000u;
}

template <int MODE>
__global__ __launch_bounds__(64) void reuse_kernel(uint32_t* out, const uint32_t* junk, int iters,
                                                   uint32_t bytes) {
  __shared__ u32x4 lj[64];
  const uint32_t lane = threadIdx.x;
  const uint32_t wave = blockIdx.x;
  lj[lane] = u32x4{0xDEAD0000u | lane, 0xDEAD1000u, 0xDEAD2000u, 0xDEAD3000u};
  __syncthreads();
  // buffer resource of out (num_records = bytes, raw buffer); its words uniform
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rj =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(junk), 0, 64 * 16, 0x00020000);
  const uint32_t lds_addr = (uint32_t)(uintptr_t)(&lj[lane]);
  for (int it = 0; it < iters; ++it) {
    const uint32_t row = (uint32_t)it;
    const uint32_t e0 = expect(wave, row, lane, 0), e1 = expect(wave, row, lane, 1);
    const uint32_t e2 = expect(wave, row, lane, 2), e3 = expect(wave, row, lane, 3);
    const uint32_t voff = ((wave * (uint32_t)iters + row) * 64u + lane) * 16u;
    const uint32_t soff = 0;
    if constexpr (MODE == 0) {
      asm volatile(
          "v_mov_b32 v40, %0\n v_mov_b32 v41, %1\n v_mov_b32 v42, %2\n v_mov_b32 v43, %3\n"
          "s_nop 4\n"
          "buffer_store_dwordx4 v[40:43], %4, %5, %6 offen\n"
          "s_nop 4\n"
          "v_mov_b32 v40, -1\n v_mov_b32 v41, -1\n v_mov_b32 v42, -1\n v_mov_b32 v43, -1\n"
          :
          : "v"(e0), "v"(e1), "v"(e2), "v"(e3), "v"(voff), "s"(r), "s"(soff)
          : "v40", "v41", "v42", "v43", "memory");
    } else if constexpr (MODE == 1) {
      asm volatile(
          "v_mov_b32 v40, %0\n v_mov_b32 v41, %1\n v_mov_b32 v42, %2\n v_mov_b32 v43, %3\n"
          "s_nop 4\n"
          "buffer_store_dwordx4 v[40:43], %4, %5, %6 offen\n"
          "v_mov_b32 v40, -1\n v_mov_b32 v41, -1\n v_mov_b32 v42, -1\n v_mov_b32 v43, -1\n"
          :
          : "v"(e0), "v"(e1), "v"(e2), "v"(e3), "v"(voff), "s"(r), "s"(soff)
          : "v40", "v41", "v42", "v43", "memory");
    } else if constexpr (MODE == 2) {
      asm volatile(
          "v_mov_b32 v40, %0\n v_mov_b32 v41, %1\n v_mov_b32 v42, %2\n v_mov_b32 v43, %3\n"
          "s_nop 4\n"
          "buffer_store_dwordx4 v[40:43], %4, %5, 0 offen\n"
          "v_mov_b32 v40, -1\n v_mov_b32 v41, -1\n v_mov_b32 v42, -1\n v_mov_b32 v43, -1\n"
          :
          : "v"(e0), "v"(e1), "v"(e2), "v"(e3), "v"(voff), "s"(r)
          : "v40", "v41", "v42", "v43", "memory");
    } else if constexpr (MODE == 3) {
      asm volatile(
          "v_mov_b32 v40, %0\n v_mov_b32 v41, %1\n v_mov_b32 v42, %2\n v_mov_b32 v43, %3\n"
          "s_nop 4\n"
          "buffer_store_dwordx4 v[40:43], %4, %5, %6 offen\n"
          "ds_read_b128 v[40:43], %7\n"
          "s_waitcnt lgkmcnt(0)\n"
          :
          : "v"(e0), "v"(e1), "v"(e2), "v"(e3), "v"(voff), "s"(r), "s"(soff), "v"(lds_addr)
          : "v40", "v41", "v42", "v43", "memory");
    } else if constexpr (MODE == 5) {
      asm volatile(
          "v_mov_b32 v40, %0\n v_mov_b32 v41, %1\n v_mov_b32 v42, %2\n v_mov_b32 v43, %3\n"
          "s_nop 4\n"
          "buffer_store_dwordx4 v[40:43], %4, %5, %6 offen\n"
          "s_nop 0\n"
          "v_mov_b32 v40, -1\n v_mov_b32 v41, -1\n v_mov_b32 v42, -1\n v_mov_b32 v43, -1\n"
          :
          : "v"(e0), "v"(e1), "v"(e2), "v"(e3), "v"(voff), "s"(r), "s"(soff)
          : "v40", "v41", "v42", "v43", "memory");
    } else if constexpr (MODE == 6) {
      asm volatile(
          "v_mov_b32 v40, %0\n v_mov_b32 v41, %1\n v_mov_b32 v42, %2\n v_mov_b32 v43, %3\n"
          "s_nop 4\n"
          "buffer_store_dwordx4 v[40:43], %4, %5, %6 offen\n"
          "v_mov_b32 v44, -1\n"
          "v_mov_b32 v40, -1\n v_mov_b32 v41, -1\n v_mov_b32 v42, -1\n v_mov_b32 v43, -1\n"
          :
          : "v"(e0), "v"(e1), "v"(e2), "v"(e3), "v"(voff), "s"(r), "s"(soff)
          : "v40", "v41", "v42", "v43", "v44", "memory");
    } else {
      asm volatile(
          "v_mov_b32 v40, %0\n v_mov_b32 v41, %1\n v_mov_b32 v42, %2\n v_mov_b32 v43, %3\n"
          "s_nop 4\n"
          "buffer_store_dwordx4 v[40:43], %4, %5, %6 offen\n"
          "buffer_load_dwordx4 v[40:43], %7, %8, 0 offen\n"
          "s_waitcnt vmcnt(0)\n"
          :
          : "v"(e0), "v"(e1), "v"(e2), "v"(e3), "v"(voff), "s"(r), "s"(soff), "v"(lane * 16u),
            "s"(rj)
          : "v40", "v41", "v42", "v43", "memory");
    }
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 64;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int waves = cus * 32;  // enough waves to keep every CU's memory pipe full
  const size_t bytes = (size_t)waves * iters * 64 * 16;
  if (bytes >= (1ull << 32)) {
    std::fprintf(stderr, "too many bytes for one buffer resource\n");
    return 2;
  }
  uint32_t *out = nullptr, *junk = nullptr;
  if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&junk, 64 * 16) != hipSuccess) return 2;
  std::vector<uint32_t> hj(64 * 4);
  for (int i = 0; i < 64 * 4; ++i) hj[i] = 0xBEEF0000u | i;
  (void)hipMemcpy(junk, hj.data(), 64 * 16, hipMemcpyHostToDevice);
  std::vector<uint32_t> h(bytes / 4);
  const char* names[] = {"nop (control)", "valu after store, SGPR soffset",
                         "valu after store, soffset 0", "ds_read into store data",
                         "buffer_load into store data", "valu after s_nop 0",
                         "valu at distance 2"};
  int rc = 0;
  for (int mode = 0; mode < 7; ++mode) {
    long bad_rows = 0, bad_words = 0;
    for (int rep = 0; rep < 4; ++rep) {
      (void)hipMemset(out, 0, bytes);
      switch (mode) {
        case 0: hipLaunchKernelGGL(reuse_kernel<0>, dim3(waves), dim3(64), 0, 0, out, junk, iters, (uint32_t)bytes); break;
        case 1: hipLaunchKernelGGL(reuse_kernel<1>, dim3(waves), dim3(64), 0, 0, out, junk, iters, (uint32_t)bytes); break;
        case 2: hipLaunchKernelGGL(reuse_kernel<2>, dim3(waves), dim3(64), 0, 0, out, junk, iters, (uint32_t)bytes); break;
        case 3: hipLaunchKernelGGL(reuse_kernel<3>, dim3(waves), dim3(64), 0, 0, out, junk, iters, (uint32_t)bytes); break;
        case 5: hipLaunchKernelGGL(reuse_kernel<5>, dim3(waves), dim3(64), 0, 0, out, junk, iters, (uint32_t)bytes); break;
        case 6: hipLaunchKernelGGL(reuse_kernel<6>, dim3(waves), dim3(64), 0, 0, out, junk, iters, (uint32_t)bytes); break;
        default: hipLaunchKernelGGL(reuse_kernel<4>, dim3(waves), dim3(64), 0, 0, out, junk, iters, (uint32_t)bytes); break;
      }
      if (hipDeviceSynchronize() != hipSuccess) {
        std::fprintf(stderr, "kernel failed\n");
        return 3;
      }
      (void)hipMemcpy(h.data(), out, bytes, hipMemcpyDeviceToHost);
      for (size_t w = 0; w < (size_t)waves; ++w)
        for (int it = 0; it < iters; ++it)
          for (uint32_t l = 0; l < 64; ++l) {
            const size_t base = (((w * iters) + it) * 64 + l) * 4;
            int bw = 0;
            for (uint32_t d = 0; d < 4; ++d) {
              const uint32_t e = ((uint32_t)w * 2654435761u) ^ ((uint32_t)it * 40503u) ^ (l << 8) ^ d ^
                                 0x5A5A0000u;
              if (h[base + d] != e) {
                if (bad_words < 3)
                  std::printf("    mode %d wave %zu row %d lane %u dword %u: got %08x want %08x\n",
                              mode, w, it, l, d, h[base + d], e);
                ++bw;
              }
            }
            bad_words += bw;
            bad_rows += bw != 0;
          }
    }
    std::printf("mode %d %-30s corrupted rows %ld / %ld, words %ld\n", mode, names[mode], bad_rows,
                (long)waves * iters * 64 * 4, bad_words);
    std::fflush(stdout);
    if (mode == 0 && bad_rows) rc = 1;  // the control must be clean
  }
  (void)hipFree(out);
  (void)hipFree(junk);
  return rc;
}
