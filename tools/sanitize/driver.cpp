// AddressSanitizer / UBSan driver for the host-side code the GPU path and
// its checker depend on (SURVEY.md §5 "sanitizers"):
//   * trex_amd/csrc/plan.cpp -- the topology planner (uniform and ragged
//     batches) on random, quirky (-1 fills, forward references, DAGs,
//     orphans), cyclic and malformed child lists, writing into buffers sized
//     exactly by trex_plan_ints / trex_ragged_plan_ints;
//   * oracle/cpu_port.c -- the OpenMP C restatement (the CPU baseline and a
//     test checker) on random trees, Q = 2..20, hard and softmin, with and
//     without the DP table output.
// Built by tools/sanitize/Makefile with -fsanitize=address,undefined
// -fno-sanitize-recover=all; any report aborts with a non-zero exit.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../include/trex_hip.h"

namespace trex {
// plan.cpp reports errors through the library's set_error (sankoff.hip)
int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  char buf[512];
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return code;
}
}  // namespace trex

extern "C" int sankoff_cpu_fwd_bwd(const int32_t* children, const int8_t* leaves,
                                   const float* cost, int B, int L, int n_all, int Q, float tau,
                                   float* dp_out, double* tree_score, double* d_cost,
                                   int want_grad, int nthreads);

namespace {

std::mt19937 rng(12345);

int rnd(int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); }

// coalescent merge: child ids below the parent (trex's numbering)
void random_tree(int nl, int32_t* ch) {
  const int n_all = 2 * nl - 1;
  for (int i = 0; i < 2 * n_all; ++i) ch[i] = -1;
  std::vector<int> active;
  for (int i = 0; i < nl; ++i) active.push_back(i);
  for (int k = 0; k < nl - 1; ++k) {
    const int a = rnd(0, (int)active.size() - 1);
    int b = rnd(0, (int)active.size() - 2);
    if (b >= a) ++b;
    const int ca = active[a], cb = active[b];
    const int parent = nl + k;
    ch[2 * parent] = std::min(ca, cb);
    ch[2 * parent + 1] = std::max(ca, cb);
    active.erase(active.begin() + std::max(a, b));
    active.erase(active.begin() + std::min(a, b));
    active.push_back(parent);
  }
}

// the quirks trex's child rule allows (sankoff.py:60,67)
void perturb(int nl, int32_t* ch, int mode) {
  const int n_all = 2 * nl - 1;
  const int node = rnd(nl, n_all - 1);
  switch (mode) {
    case 0: ch[2 * node + 1] = -1; break;                       // -1 fill
    case 1: ch[2 * node] = rnd(node, n_all - 1); break;         // forward ref / self
    case 2: ch[2 * node] = rnd(nl, std::max(nl, node - 1)); break;  // DAG / orphan
    case 3: ch[2 * node] = n_all + 3; break;                    // malformed (rejected)
    default: break;
  }
}

int check_uniform() {
  int runs = 0;
  for (int it = 0; it < 400; ++it) {
    const int nl = rnd(2, 128);
    const int n_all = 2 * nl - 1;
    const int B = rnd(1, 6);
    std::vector<int32_t> ch((size_t)B * n_all * 2);
    for (int b = 0; b < B; ++b) {
      random_tree(nl, ch.data() + (size_t)b * n_all * 2);
      if (it % 2) perturb(nl, ch.data() + (size_t)b * n_all * 2, rnd(0, 4));
    }
    const int64_t n = trex_plan_ints(B, n_all);
    if (n <= 0) continue;  // n_all < 3 is rejected by trex_plan_ints / trex_plan_build
    std::vector<int32_t> plan((size_t)n);
    int32_t info[4];
    const int rc = trex_plan_build(ch.data(), B, n_all, plan.data(), info);
    if (rc != 0 && rc != TREX_E_TOPOLOGY && rc != TREX_E_ARG) return 1;
    ++runs;
  }
  std::printf("uniform plans: %d\n", runs);
  return 0;
}

int check_ragged() {
  for (int it = 0; it < 200; ++it) {
    const int B = rnd(1, 8);
    std::vector<int32_t> n_all(B), L(B);
    size_t tot = 0;
    for (int b = 0; b < B; ++b) {
      n_all[b] = 2 * rnd(2, 70) - 1;
      L[b] = rnd(1, 700);
      tot += (size_t)n_all[b] * 2;
    }
    std::vector<int32_t> ch(tot);
    size_t off = 0;
    for (int b = 0; b < B; ++b) {
      const int nl = (n_all[b] + 1) / 2;
      random_tree(nl, ch.data() + off);
      if (it % 3 == 0) perturb(nl, ch.data() + off, rnd(0, 4));
      off += (size_t)n_all[b] * 2;
    }
    const int64_t n = trex_ragged_plan_ints(B, n_all.data(), L.data());
    if (n <= 0) return 2;
    std::vector<int32_t> plan((size_t)n);
    int64_t info[8];
    const int rc = trex_ragged_plan_build(ch.data(), n_all.data(), L.data(), B, plan.data(), info);
    if (rc != 0 && rc != TREX_E_TOPOLOGY && rc != TREX_E_ARG) return 3;
  }
  std::printf("ragged plans: 200\n");
  return 0;
}

int check_cpu_port() {
  for (int it = 0; it < 24; ++it) {
    const int nl = rnd(2, 40);
    const int n_all = 2 * nl - 1;
    const int B = rnd(1, 3);
    const int L = rnd(1, 300);
    const int Q = rnd(2, 20);
    const float tau = (it % 2) ? 0.0f : 0.5f;
    std::vector<int32_t> ch((size_t)B * n_all * 2);
    for (int b = 0; b < B; ++b) random_tree(nl, ch.data() + (size_t)b * n_all * 2);
    std::vector<int8_t> leaves((size_t)B * nl * L);
    for (auto& x : leaves) x = (int8_t)rnd(-1, Q);  // -1 / Q: missing (all-1e5 row)
    std::vector<float> cost((size_t)Q * Q);
    for (int i = 0; i < Q; ++i)
      for (int j = 0; j < Q; ++j) cost[(size_t)i * Q + j] = i == j ? 0.0f : (float)rnd(1, 4);
    const int ni = n_all - nl;
    std::vector<float> dp((it % 3) ? (size_t)B * ni * Q * L : 0);
    std::vector<double> ts(B), dc((size_t)Q * Q);
    const int rc = sankoff_cpu_fwd_bwd(ch.data(), leaves.data(), cost.data(), B, L, n_all, Q, tau,
                                       dp.empty() ? nullptr : dp.data(), ts.data(), dc.data(),
                                       1, 2);
    if (rc != 0) return 4;
  }
  std::printf("cpu port runs: 24\n");
  return 0;
}

}  // namespace

int main() {
  if (int e = check_uniform()) return e;
  if (int e = check_ragged()) return e;
  if (int e = check_cpu_port()) return e;
  std::printf("sanitize ok\n");
  return 0;
}
