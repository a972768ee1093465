// libtrexhip.so -- trex's raw-table Sankoff entry points on MI355X (gfx950):
// run_dp / vectorized_dp and backtrack_sankoff_jit operating directly on the
// reference's own tables (maraxen/trex src/trex/sankoff.py:24-97, 191-267):
//
//   DP table            fp32 [L][n_all][Q]     (VmappedDPTable, utils/types.py:53)
//   backtracking table  fp32 [L][n_all][Q][4]  (BacktrackingTable, :56; per
//                       node and parent state: child 1 id, child 1 state,
//                       child 2 id, child 2 state, stored as floats)
//
// These are the drop-in for callers that hold the tables themselves (the
// reference's tests/test_sankoff.py:31 calls run_dp with a caller-initialised
// table).  The engine kernels (sankoff.hip / sankoff_wide.hip) never build the
// backtracking table -- they re-derive argmins from the DP rows -- so the
// batched hot path does not go through here.
//
// Semantics restated from the reference, including what a caller-supplied
// table makes observable:
//   * leaf rows i < (n_all+1)//2 keep the caller's values except
//     dp[i, int(seq)] = 0 (truncation toward zero, negative wraps once,
//     anything else out of range is a dropped scatter, :49-52);
//   * nodes n_leaves..n_all-1 in index order (:87-92); children = the first
//     two rows with adj[row, node] == 1, -1 filled (:60, computed on the host
//     without run_sankoff's root self-loop removal, which run_dp does not do);
//     child -1 reads the last row; a child row not yet written holds the
//     caller's value at the time it is read;
//   * per child: min_j and FIRST argmin_j of C[i][j] + dp[c][j] with jnp's NaN
//     rules (min propagates NaN; argmin picks the first NaN), accumulated
//     0 + m1 + m2 (:62-77); dp[node] and bt[node] overwritten (:79-83);
//   * backtrack: the reference's explicit stack of n_all (node, state) int32
//     pairs, popped while non-empty; ancestors (node >= n_leaves) record their
//     state and push both children from bt (float -> int32 truncation);
//     gathers clamp (negative state indices wrap first), scatters beyond the
//     stack / output drop (:212-265).  A table whose DFS does not terminate
//     (the reference hangs) stops after max_steps pops and reports it.
//
// This translation unit is compiled WITHOUT -fno-honor-nans (Makefile): a
// caller's table may hold NaN, and the NaN rules above are part of the
// contract.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "trex_common.h"

namespace trex {

namespace {

constexpr int kRdThreads = 256;

__device__ __forceinline__ bool is_nan(float x) { return x != x; }

// jnp.min / jnp.argmin over j of row_i[j] + d[j] (XLA reduce semantics:
// NaN propagates; argmin = first NaN if any, else first minimum)
struct MinArg {
  float v;
  int j;
};

// trex leaf code: XLA's f32 -> s32 convert (truncation, saturation, NaN -> 0),
// negative wraps once, -1 = dropped
__device__ __forceinline__ int leaf_state(float x, int Q) {
  if (is_nan(x)) return 0;
  if (!(x > -2147483648.0f && x < 2147483648.0f)) return -1;  // saturated: out of range, dropped
  int s = (int)x;  // truncation toward zero
  if (s < 0) s += Q;
  return (s >= 0 && s < Q) ? s : -1;
}

// QMAX > 0: child rows in registers (Q <= QMAX); QMAX == 0: any Q, rows
// re-read from the (L1/L2-resident) table
template <int QMAX>
__global__ __launch_bounds__(kRdThreads) void run_dp_kernel(
    const int32_t* __restrict__ children, int n_all, int nl, int L, int Q,
    const float* __restrict__ seqs, int n_codes, const float* __restrict__ cost, int cost_in_lds,
    float* __restrict__ dp, float* __restrict__ bt) {
  extern __shared__ float cl[];  // C [Q][Q] when it fits
  if (cost_in_lds)
    for (int t = threadIdx.x; t < Q * Q; t += kRdThreads) cl[t] = cost[t];
  __syncthreads();
  const float* C = cost_in_lds ? cl : cost;
  const int l = blockIdx.x * kRdThreads + threadIdx.x;
  if (l >= L) return;
  const size_t row = (size_t)Q;
  float* D = dp + (size_t)l * n_all * row;
  float4* BT = reinterpret_cast<float4*>(bt + (size_t)l * n_all * row * 4);
  // leaf init (sankoff.py:49-52): seqs [n_seq][n_codes][L]
  for (int i = 0; i < nl; ++i)
    for (int c = 0; c < n_codes; ++c) {
      const int s = leaf_state(seqs[((size_t)i * n_codes + c) * L + l], Q);
      if (s >= 0) D[(size_t)i * row + s] = 0.0f;
    }
  for (int node = nl; node < n_all; ++node) {
    const int c0 = children[2 * node], c1 = children[2 * node + 1];
    const int r0 = c0 < 0 ? c0 + n_all : c0;  // jnp gather: -1 wraps to the last row
    const int r1 = c1 < 0 ? c1 + n_all : c1;
    if constexpr (QMAX > 0) {
      float d0[QMAX], d1[QMAX];
#pragma unroll
      for (int j = 0; j < QMAX; ++j) {
        d0[j] = j < Q ? D[(size_t)r0 * row + j] : 0.0f;
        d1[j] = j < Q ? D[(size_t)r1 * row + j] : 0.0f;
      }
      // both child rows are in registers before the node's rows are written,
      // so a node listed as its own child reads its old row (:67 before :79)
      for (int i = 0; i < Q; ++i) {
        MinArg m0{C[i * Q] + d0[0], 0}, m1{C[i * Q] + d1[0], 0};
#pragma unroll
        for (int j = 1; j < QMAX; ++j) {
          if (j < Q) {
            const float v0 = C[i * Q + j] + d0[j], v1 = C[i * Q + j] + d1[j];
            if (v0 < m0.v || (is_nan(v0) && !is_nan(m0.v))) m0 = MinArg{v0, j};
            if (v1 < m1.v || (is_nan(v1) && !is_nan(m1.v))) m1 = MinArg{v1, j};
          }
        }
        D[(size_t)node * row + i] = (0.0f + m0.v) + m1.v;  // scan carry from zeros (:73-77)
        BT[(size_t)node * row + i] = make_float4((float)c0, (float)m0.j, (float)c1, (float)m1.j);
      }
    } else {
      // any Q, rows re-read from the table.  A node listed as its own child
      // reads its old row (:67 reads before :79 writes): its results are
      // staged in its bt row (never read by the DP) and moved afterwards.
      const bool self = (r0 == node) || (r1 == node);
      for (int i = 0; i < Q; ++i) {
        const float* ci = C + (size_t)i * Q;
        MinArg m0{ci[0] + D[(size_t)r0 * row], 0}, m1{ci[0] + D[(size_t)r1 * row], 0};
        for (int j = 1; j < Q; ++j) {
          const float v0 = ci[j] + D[(size_t)r0 * row + j];
          const float v1 = ci[j] + D[(size_t)r1 * row + j];
          if (v0 < m0.v || (is_nan(v0) && !is_nan(m0.v))) m0 = MinArg{v0, j};
          if (v1 < m1.v || (is_nan(v1) && !is_nan(m1.v))) m1 = MinArg{v1, j};
        }
        const float tot = (0.0f + m0.v) + m1.v;
        if (self) {
          BT[(size_t)node * row + i] = make_float4(tot, (float)m0.j, 0.0f, (float)m1.j);
        } else {
          D[(size_t)node * row + i] = tot;
          BT[(size_t)node * row + i] = make_float4((float)c0, (float)m0.j, (float)c1, (float)m1.j);
        }
      }
      if (self)
        for (int i = 0; i < Q; ++i) {
          const float4 v = BT[(size_t)node * row + i];
          D[(size_t)node * row + i] = v.x;
          BT[(size_t)node * row + i] = make_float4((float)c0, v.y, (float)c1, v.w);
        }
    }
  }
}

// float -> int32 as XLA's convert (truncation; NaN -> 0, saturating)
__device__ __forceinline__ int f2i(float x) {
  if (is_nan(x)) return 0;
  if (x >= 2147483647.0f) return 2147483647;
  if (x <= -2147483648.0f) return (int)0x80000000;
  return (int)x;
}

// vmap(backtrack_sankoff_jit) over sites (sankoff.py:166-180, 191-267).
// stack [n_all][L] int2 (site-innermost: lanes at the same depth coalesce),
// out [n_all][L] int32.
// root_state NULL: the root state is jnp.argmin(dp[:, root_node, :], axis=1)
// (sankoff.py:172; first minimum, first NaN), read from dp [L][n_all][Q].
__global__ __launch_bounds__(kRdThreads) void backtrack_generic_kernel(
    int root_node, const int32_t* __restrict__ root_state, const float* __restrict__ dp,
    const float* __restrict__ bt, int n_all, int n_leaves, int L, int Q, int2* __restrict__ stack,
    int32_t* __restrict__ out, int64_t max_steps, int32_t* __restrict__ status) {
  const int l = blockIdx.x * kRdThreads + threadIdx.x;
  if (l >= L) return;
  for (int k = 0; k < n_all; ++k) {
    stack[(size_t)k * L + l] = make_int2(0, 0);
    out[(size_t)k * L + l] = 0;
  }
  int rs;
  if (root_state) {
    rs = root_state[l];
  } else {
    const int rn = min(max(root_node < 0 ? root_node + n_all : root_node, 0), n_all - 1);
    const float* d = dp + ((size_t)l * n_all + rn) * Q;
    MinArg m{d[0], 0};
    for (int j = 1; j < Q; ++j)
      if (d[j] < m.v || (is_nan(d[j]) && !is_nan(m.v))) m = MinArg{d[j], j};
    rs = m.j;
  }
  stack[l] = make_int2(root_node, rs);
  const float4* B = reinterpret_cast<const float4*>(bt + (size_t)l * n_all * Q * 4);
  int ptr = 1;
  int64_t steps = 0;
  while (ptr > 0) {
    if (++steps > max_steps) {
      atomicOr(status, 1);
      return;
    }
    const int cur = ptr - 1;
    const int2 e = stack[(size_t)min(cur, n_all - 1) * L + l];  // gather clamps
    const int node = e.x, state = e.y;
    if (node >= n_leaves) {
      if (node < n_all) out[(size_t)node * L + l] = state;  // scatter drops
      int s = state < 0 ? state + Q : state;
      s = min(max(s, 0), Q - 1);
      const int nd = min(node, n_all - 1);
      const float4 ci = B[(size_t)nd * Q + s];
      if (cur < n_all) stack[(size_t)cur * L + l] = make_int2(f2i(ci.x), f2i(ci.y));
      if (cur + 1 < n_all) stack[(size_t)(cur + 1) * L + l] = make_int2(f2i(ci.z), f2i(ci.w));
      ptr = cur + 2;
    } else {
      ptr = cur;
    }
  }
}

// run_sankoff's total over a raw table (sankoff.py:187: dp[:, -1].min(axis=1)
// .sum(); jnp.min propagates NaN): per-site minimum of the root row, then one
// workgroup sums the minima in fp64 in a fixed order (thread t: sites t,
// t + 256, ...; then a fixed LDS tree) and rounds once to fp32
__global__ __launch_bounds__(kRdThreads) void root_min_kernel(const float* __restrict__ dp, int L,
                                                             int n_all, int Q,
                                                             float* __restrict__ site_min) {
  const int l = blockIdx.x * kRdThreads + threadIdx.x;
  if (l >= L) return;
  const float* d = dp + ((size_t)l * n_all + (n_all - 1)) * Q;
  float m = d[0];
  for (int j = 1; j < Q; ++j)
    if (d[j] < m || is_nan(d[j])) m = d[j];
  site_min[l] = m;
}

__global__ __launch_bounds__(kRdThreads) void root_total_kernel(const float* __restrict__ site_min,
                                                               int L, float* __restrict__ total) {
  __shared__ double part[kRdThreads];
  double s = 0.0;
  for (int l = threadIdx.x; l < L; l += kRdThreads) s += (double)site_min[l];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = kRdThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = (float)part[0];
}

int rd_check(const char* fn) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TREX_E_HIP, "%s: %s", fn, hipGetErrorString(e));
  return TREX_OK;
}

}  // namespace
}  // namespace trex

using namespace trex;

extern "C" int trex_run_dp(const int32_t* children, int n_all, int L, int Q, const float* seqs,
                           int n_codes, const float* cost, float* dp, float* bt, void* stream) {
  const char* fn = "trex_run_dp";
  if (n_all < 1 || L <= 0 || Q < 1 || n_codes < 0 || !children || !cost || !dp || !bt ||
      (n_codes > 0 && !seqs))
    return set_error(TREX_E_ARG, "%s: bad arguments (n_all=%d L=%d Q=%d)", fn, n_all, L, Q);
  if ((int64_t)L * n_all * Q * 4 > ((int64_t)1 << 40))
    return set_error(TREX_E_ARG, "%s: table too large", fn);
  const int nl = (n_all + 1) / 2;
  const size_t cbytes = (size_t)Q * Q * 4;
  const int in_lds = cbytes <= 65536 ? 1 : 0;
  const size_t lds = in_lds ? cbytes : 0;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((L + kRdThreads - 1) / kRdThreads);
#define TREX_RD(QM)                                                                             \
  hipLaunchKernelGGL(run_dp_kernel<QM>, grid, dim3(kRdThreads), lds, st, children, n_all, nl, L, \
                     Q, seqs, n_codes, cost, in_lds, dp, bt)
  if (Q <= 4) TREX_RD(4);
  else if (Q <= 8) TREX_RD(8);
  else if (Q <= 16) TREX_RD(16);
  else if (Q <= 32) TREX_RD(32);
  else TREX_RD(0);
#undef TREX_RD
  return rd_check(fn);
}

extern "C" int64_t trex_backtrack_workspace_bytes(int n_all, int L) {
  if (n_all < 1 || L <= 0) return 0;
  return (int64_t)n_all * L * 8;
}

extern "C" int trex_backtrack_generic(int root_node, const int32_t* root_state, const float* dp,
                                      const float* bt, int n_all, int n_leaves, int L, int Q,
                                      int32_t* out, void* stack_ws, int64_t stack_bytes,
                                      int64_t max_steps, int32_t* status, void* stream) {
  const char* fn = "trex_backtrack_generic";
  if (n_all < 1 || L <= 0 || Q < 1 || (!root_state && !dp) || !bt || !out || !stack_ws ||
      !status || max_steps <= 0)
    return set_error(TREX_E_ARG, "%s: bad arguments", fn);
  if (stack_bytes < trex_backtrack_workspace_bytes(n_all, L))
    return set_error(TREX_E_ARG, "%s: stack workspace too small", fn);
  hipLaunchKernelGGL(backtrack_generic_kernel, dim3((L + kRdThreads - 1) / kRdThreads),
                     dim3(kRdThreads), 0, (hipStream_t)stream, root_node, root_state, dp, bt, n_all,
                     n_leaves, L, Q, static_cast<int2*>(stack_ws), out, max_steps, status);
  return rd_check(fn);
}

extern "C" int trex_dp_root_total(const float* dp, int L, int n_all, int Q, float* site_min,
                                  float* total, void* stream) {
  const char* fn = "trex_dp_root_total";
  if (n_all < 1 || L <= 0 || Q < 1 || !dp || !site_min || !total)
    return set_error(TREX_E_ARG, "%s: bad arguments (n_all=%d L=%d Q=%d)", fn, n_all, L, Q);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(root_min_kernel, dim3((L + kRdThreads - 1) / kRdThreads), dim3(kRdThreads), 0,
                     st, dp, L, n_all, Q, site_min);
  hipLaunchKernelGGL(root_total_kernel, dim3(1), dim3(kRdThreads), 0, st, site_min, L, total);
  return rd_check(fn);
}
