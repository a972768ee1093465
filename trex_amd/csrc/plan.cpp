// Host-side topology planner for libtrexhip.so.
//
// Turns trex's per-node child lists (jnp.where(adj[:, node] == 1, size=2,
// fill_value=-1), src/trex/sankoff.py:60) into a per-tree "program" the HIP
// kernels execute with wave-uniform control flow:
//
//  * forward steps in a post-order that evaluates the child needing more
//    stack slots first (Sethi-Ullman), so live internal DP vectors fit a
//    log2(n)+1-deep per-lane LDS stack instead of being re-read from HBM;
//  * the child rules of trex's run_dp: c == -1 or c >= node reads a row that
//    still holds the 1e5 init (sankoff.py:60,67,152), c < n_leaves is a leaf,
//    otherwise an already computed internal row;
//  * adjoint flags for the reverse sweep (which reverse step first writes a
//    child's cotangent slot, which nodes the root never reaches);
//  * the reference backtrack's visiting order (sankoff.py:212-265), simulated
//    once on the topology (the DFS node sequence does not depend on states),
//    reduced to "node x takes its state from parent p at x's last visit".
//
// This is integer work on B * n_all entries, done once per topology (the
// reference re-traces per static shape, sankoff.py:114).
#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <functional>
#include <queue>
#include <set>
#include <vector>

#include "trex_common.h"

namespace trex {

namespace {

constexpr int kKindSent = 0, kKindLeaf = 1, kKindInt = 2;

struct Child {
  int kind;
  int index;  // leaf index or internal row
};

// One tree.  Returns false on a malformed child id.
bool plan_one_tree(const int32_t* ch, int n_all, int32_t* fwd, int32_t* bt,
                   int* n_slots, int* bt_ok, int* n_dag, int* n_unreached) {
  const int nl = (n_all + 1) / 2;
  const int ni = n_all - nl;
  std::vector<Child> kids(2 * ni);
  std::vector<int> refs(ni, 0);
  for (int r = 0; r < ni; ++r) {
    const int node = nl + r;
    for (int k = 0; k < 2; ++k) {
      const int c = ch[2 * node + k];
      if (c < -1 || c >= n_all) return false;
      Child cd;
      if (c == -1 || c >= node) {
        cd = {kKindSent, 0};
      } else if (c < nl) {
        cd = {kKindLeaf, c};
      } else {
        cd = {kKindInt, c - nl};
        refs[c - nl] += 1;
      }
      kids[2 * r + k] = cd;
    }
  }
  int dag = 0;
  for (int r = 0; r < ni; ++r) dag += refs[r] > 1;
  *n_dag = dag;

  // Sethi-Ullman need, rows in increasing order (internal children are lower)
  std::vector<int> need(ni, 1);
  for (int r = 0; r < ni; ++r) {
    int a = 0, b = 0;
    for (int k = 0; k < 2; ++k) {
      const Child& cd = kids[2 * r + k];
      if (cd.kind == kKindInt) {
        const int n = need[cd.index];
        if (n > a) { b = a; a = n; } else if (n > b) { b = n; }
      }
    }
    need[r] = std::max({1, a, b + 1});
  }

  // schedule: post-order DFS, heavier child first; orphans first, root last
  std::vector<int> order;
  order.reserve(ni);
  std::vector<char> done(ni, 0);
  auto visit = [&](int start) {
    std::vector<std::pair<int, int>> st;  // (row, phase)
    st.push_back({start, 0});
    while (!st.empty()) {
      auto [r, ph] = st.back();
      st.pop_back();
      if (done[r]) continue;
      if (ph == 1) {
        done[r] = 1;
        order.push_back(r);
        continue;
      }
      st.push_back({r, 1});
      int c0 = -1, c1 = -1;
      if (kids[2 * r].kind == kKindInt) c0 = kids[2 * r].index;
      if (kids[2 * r + 1].kind == kKindInt) c1 = kids[2 * r + 1].index;
      // push the lighter first so the heavier is evaluated first
      int heavy = c0, light = c1;
      if (c0 < 0 || (c1 >= 0 && need[c1] > need[c0])) { heavy = c1; light = c0; }
      if (light >= 0 && !done[light]) st.push_back({light, 0});
      if (heavy >= 0 && !done[heavy]) st.push_back({heavy, 0});
    }
  };
  for (int r = 0; r < ni - 1; ++r)
    if (refs[r] == 0) visit(r);
  visit(ni - 1);
  if ((int)order.size() != ni) return false;  // unreachable in a DAG of lower ids

  // register bypass: in this post-order the step right before a node is its
  // last-evaluated child; when that child has no other consumer its vector
  // never needs a slot (forward D, adjoint cotangent stay in registers)
  std::vector<int> pos(ni, 0), consumer(ni, -1);
  for (int k = 0; k < ni; ++k) pos[order[k]] = k;
  for (int r = 0; r < ni; ++r)
    for (int k = 0; k < 2; ++k)
      if (kids[2 * r + k].kind == kKindInt) consumer[kids[2 * r + k].index] = r;
  std::vector<char> bypass(ni, 0);
  for (int r = 0; r < ni; ++r)
    bypass[r] = refs[r] == 1 && consumer[r] >= 0 && pos[consumer[r]] == pos[r] + 1;

  // slot simulation (bypassed vectors take no slot)
  std::vector<int> remaining(refs), slot(ni, 0xFF);
  std::set<int> free_slots;
  int top = 0, maxs = 0;
  for (int r : order) {
    for (int k = 0; k < 2; ++k) {
      const Child& cd = kids[2 * r + k];
      if (cd.kind != kKindInt || bypass[cd.index]) continue;
      if (--remaining[cd.index] == 0) free_slots.insert(slot[cd.index]);
    }
    if (refs[r] > 0 && !bypass[r]) {
      int s;
      if (!free_slots.empty()) {
        s = *free_slots.begin();
        free_slots.erase(free_slots.begin());
      } else {
        s = top++;
      }
      slot[r] = s;
      maxs = std::max(maxs, s + 1);
    }
  }
  if (maxs > 250) return false;
  *n_slots = maxs;

  // reachability from the root along real internal edges (adjoint support)
  std::vector<char> reach(ni, 0);
  reach[ni - 1] = 1;
  for (int r = ni - 1; r >= 0; --r) {
    if (!reach[r]) continue;
    for (int k = 0; k < 2; ++k)
      if (kids[2 * r + k].kind == kKindInt) reach[kids[2 * r + k].index] = 1;
  }
  int unr = 0;
  for (int r = 0; r < ni; ++r) unr += !reach[r];
  *n_unreached = unr;

  // deferred edges (kChildDeferred): cherries with one reached parent
  // (TREX_DEFER=0 turns them off, A/B)
  static const bool defer_on = [] {
    const char* e = std::getenv("TREX_DEFER");
    return !(e && e[0] == '0');
  }();
  std::vector<char> deferred(ni, 0);
  if (defer_on)
    for (int c = 0; c < ni; ++c)
      deferred[c] = refs[c] == 1 && consumer[c] >= 0 && reach[consumer[c]] &&
                    kids[2 * c].kind != kKindInt && kids[2 * c + 1].kind != kKindInt;

  // encode forward steps; set/accumulate flags follow the reverse order
  std::vector<char> seen(ni, 0);
  std::vector<int32_t> enc(4 * ni);
  for (int k = ni - 1; k >= 0; --k) {
    const int r = order[k];
    int32_t* e = &enc[4 * k];
    e[0] = (r & 0xFFFF) | ((slot[r] & 0xFF) << 16);
    for (int j = 0; j < 2; ++j) {
      const Child& cd = kids[2 * r + j];
      int32_t d = (cd.index & 0xFFFF) | (cd.kind << 24);
      if (cd.kind == kKindInt) {
        d |= (slot[cd.index] & 0xFF) << 16;
        if (bypass[cd.index]) d |= kChildPrev;
        if (deferred[cd.index]) d |= kChildDeferred;
        if (reach[r]) {
          if (seen[cd.index]) d |= kStepAccumulate;
          seen[cd.index] = 1;
        }
      }
      e[1 + j] = d;
    }
    int32_t f = 0;
    if (r == ni - 1) f |= kStepRoot;
    if (!reach[r]) f |= kStepUnreached;
    if (bypass[r]) f |= kStepToNext;
    if (deferred[r]) f |= kStepDeferredIn;
    e[3] = f;
  }
  if (order.back() != ni - 1) return false;
  std::memcpy(fwd, enc.data(), enc.size() * sizeof(int32_t));

  // ---- reference backtrack simulation (sankoff.py:212-265) ----
  // stack of node ids; last_parent[x] / last_slot[x] at x's LAST visit.
  std::vector<int> last_parent(ni, -1), last_slot(ni, -1);
  std::vector<char> visited(ni, 0);
  std::vector<std::pair<int, int>> stk;  // (node, parent*2+slot) ; parent -1 = root entry
  stk.push_back({n_all - 1, -1});
  int64_t steps = 0;
  const int64_t cap = 1LL << 22;
  bool ok = true;
  while (!stk.empty()) {
    if (++steps > cap || (int64_t)stk.size() > 4LL * n_all) { ok = false; break; }
    auto [node, from] = stk.back();
    stk.pop_back();
    if (node < nl) continue;  // leaves and the -1 fill are skipped
    const int x = node - nl;
    visited[x] = 1;
    if (from >= 0) { last_parent[x] = from >> 1; last_slot[x] = from & 1; }
    const int c0 = ch[2 * node], c1 = ch[2 * node + 1];
    if (c0 == node || c1 == node) { ok = false; break; }  // self loop: never terminates
    stk.push_back({c0, 2 * x + 0});
    stk.push_back({c1, 2 * x + 1});
  }
  *bt_ok = ok ? 1 : 0;
  // process order: BFS over last-parent forest from the root
  std::vector<std::vector<int>> kidsbt(ni);
  for (int x = 0; x < ni; ++x)
    if (ok && visited[x] && last_parent[x] >= 0) kidsbt[last_parent[x]].push_back(x);
  std::vector<int32_t> benc(2 * ni, 0);
  int w = 0;
  if (ok) {
    std::queue<int> q;
    q.push(ni - 1);
    std::vector<char> emitted(ni, 0);
    while (!q.empty()) {
      const int x = q.front();
      q.pop();
      if (emitted[x]) continue;
      emitted[x] = 1;
      int kind, parent = 0;
      if (x == ni - 1) {
        kind = kBtRoot;
      } else {
        parent = last_parent[x];
        const int raw = ch[2 * (nl + parent) + last_slot[x]];
        // the parent's forward used the real row only when raw < parent node
        kind = (raw < nl + parent) ? kBtReal : kBtSentinel;
      }
      benc[2 * w] = (x & 0xFFFF) | (kind << 16) | (last_slot[x] > 0 ? (1 << 20) : 0);
      benc[2 * w + 1] = parent;
      ++w;
      for (int c : kidsbt[x]) q.push(c);
    }
    for (int x = 0; x < ni; ++x) {
      if (!emitted[x]) {
        benc[2 * w] = (x & 0xFFFF) | (kBtUnreached << 16);
        benc[2 * w + 1] = 0;
        ++w;
      }
    }
  }
  std::memcpy(bt, benc.data(), benc.size() * sizeof(int32_t));
  return true;
}

// Staged program of one tree (layout: trex_common.h).  Nodes are levelled by
// height over real internal edges (a leaf / 1e5-row child adds nothing), each
// level is one stage, its nodes dealt round-robin to the workgroup's waves:
// a stage's nodes depend only on earlier stages, so the waves run them in
// parallel and the serial chain is the tree height (6 for a balanced
// 64-taxon tree instead of 63 nodes).  A topology with a shared internal
// child (trex's DAG quirk) runs serially on wave 0 in index order, where the
// accumulate flags order its cotangent sums exactly as the single-wave
// kernels do.
void stage_one_tree(const int32_t* ch, int n_all, int32_t* region) {
  const int nl = (n_all + 1) / 2;
  const int ni = n_all - nl;
  constexpr int W = kStageWaves;
  std::vector<int> kind(2 * ni), idx(2 * ni), refs(ni, 0), height(ni, 1);
  for (int r = 0; r < ni; ++r) {
    const int node = nl + r;
    for (int k = 0; k < 2; ++k) {
      const int c = ch[2 * node + k];  // validated by plan_one_tree
      if (c == -1 || c >= node) {
        kind[2 * r + k] = kKindSent;
        idx[2 * r + k] = 0;
      } else if (c < nl) {
        kind[2 * r + k] = kKindLeaf;
        idx[2 * r + k] = c;
      } else {
        kind[2 * r + k] = kKindInt;
        idx[2 * r + k] = c - nl;
        refs[c - nl] += 1;
        height[r] = std::max(height[r], height[c - nl] + 1);
      }
    }
  }
  const bool dag = std::any_of(refs.begin(), refs.end(), [](int v) { return v > 1; });
  std::vector<char> reach(ni, 0);
  reach[ni - 1] = 1;
  for (int r = ni - 1; r >= 0; --r)
    if (reach[r])
      for (int k = 0; k < 2; ++k)
        if (kind[2 * r + k] == kKindInt) reach[idx[2 * r + k]] = 1;
  // (stage, wave) of every row
  int S = 1;
  std::vector<int> stage(ni, 0), wave(ni, 0);
  if (!dag) {
    S = *std::max_element(height.begin(), height.end());
    std::vector<int> fill(S, 0);
    for (int r = 0; r < ni; ++r) {
      stage[r] = height[r] - 1;
      wave[r] = fill[stage[r]]++ % W;
    }
  }
  std::vector<int> order(ni);
  for (int r = 0; r < ni; ++r) order[r] = r;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
    return stage[x] != stage[y] ? stage[x] < stage[y] : wave[x] < wave[y];
  });
  int32_t* steps = region;
  int32_t* offs = region + 4LL * ni + 1;
  region[4LL * ni] = S;
  for (int j = 0; j <= S * W; ++j) offs[j] = ni;
  for (int k = ni - 1; k >= 0; --k) offs[stage[order[k]] * W + wave[order[k]]] = k;
  for (int j = S * W - 1; j >= 0; --j) offs[j] = std::min(offs[j], offs[j + 1]);
  // accumulate flags follow the adjoint's order: stages, then steps, reversed
  std::vector<char> seen(ni, 0);
  for (int k = ni - 1; k >= 0; --k) {
    const int r = order[k];
    int32_t* e = steps + 4LL * k;
    e[0] = r & 0xFFFF;
    for (int j = 0; j < 2; ++j) {
      int32_t d = (idx[2 * r + j] & 0xFFFF) | (kind[2 * r + j] << 24);
      if (kind[2 * r + j] == kKindInt && reach[r]) {
        if (seen[idx[2 * r + j]]) d |= kStepAccumulate;
        seen[idx[2 * r + j]] = 1;
      }
      e[1 + j] = d;
    }
    e[3] = (r == ni - 1 ? kStepRoot : 0) | (reach[r] ? 0 : kStepUnreached);
  }
}

// Lane-per-site program of one tree (layout: trex_common.h).  Internal rows
// of height <= 2 (height: 1 + the tallest internal child; leaves and 1e5
// rows 0) are computed inline by the task that consumes them; every other
// row (and the root) is a task.  A task's stage is its height - 3 (the
// root's at least 0), so a stage depends only on earlier stages.  A task
// row's LDS slot holds its D from its own stage to its parent's (the root's:
// its own stage), then, in the reversed adjoint, its cotangent over the same
// interval: slots are
// interval-coloured, reused once the interval has ended.  Returns the slot
// count, or -1 when the tree cannot run this program (a shared internal
// child -- trex's DAG quirk --, an internal row the root does not reach, or
// more than 255 slots); the other kernels then serve the batch.
int lane_program_one_tree(const int32_t* ch, int n_all, int32_t* region) {
  const int nl = (n_all + 1) / 2;
  const int ni = n_all - nl;
  std::memset(region, 0, sizeof(int32_t) * lp_tree_ints(ni));
  region[1] = -1;
  std::vector<int> kind(2 * ni), idx(2 * ni), refs(ni, 0), height(ni, 1), parent(ni, -1);
  for (int r = 0; r < ni; ++r) {
    const int node = nl + r;
    for (int k = 0; k < 2; ++k) {
      const int c = ch[2 * node + k];  // validated by plan_one_tree
      if (c == -1 || c >= node) {
        kind[2 * r + k] = kKindSent;
        idx[2 * r + k] = 0;
      } else if (c < nl) {
        kind[2 * r + k] = kKindLeaf;
        idx[2 * r + k] = c;
      } else {
        kind[2 * r + k] = kKindInt;
        idx[2 * r + k] = c - nl;
        refs[c - nl] += 1;
        parent[c - nl] = r;
        height[r] = std::max(height[r], height[c - nl] + 1);
      }
    }
  }
  const int root = ni - 1;
  for (int r = 0; r < ni; ++r)
    if (refs[r] > 1 || (r != root && refs[r] == 0)) return -1;  // DAG / unreached row
  std::vector<char> task(ni, 0);
  std::vector<int> stage(ni, 0);
  int S = 1;
  for (int r = 0; r < ni; ++r) {
    task[r] = r == root || height[r] >= 3;
    stage[r] = std::max(0, height[r] - 3);
    if (task[r]) S = std::max(S, stage[r] + 1);
  }
  // slots: interval colouring over [stage(r), stage(parent(r))]
  std::vector<int> order;
  for (int r = 0; r < ni; ++r)
    if (task[r]) order.push_back(r);
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return stage[x] < stage[y]; });
  std::vector<int> slot(ni, 0xFF), slot_end;
  for (int r : order) {
    const int st = stage[r], en = r == root ? stage[r] : stage[parent[r]];
    int s = 0;
    while (s < (int)slot_end.size() && slot_end[s] >= st) ++s;
    if (s == (int)slot_end.size()) slot_end.push_back(en);
    else slot_end[s] = en;
    slot[r] = s;
  }
  const int n_slots = (int)slot_end.size();
  if (n_slots > 255) return -1;
  // inline rows in post-order of their task (children first): index list
  std::vector<int> inl(ni, -1);
  std::vector<int32_t> ient;
  std::function<int32_t(int, int)> desc = [&](int r, int k) -> int32_t {
    const int kd = kind[2 * r + k], c = idx[2 * r + k];
    if (kd == kKindSent) return 0;
    if (kd == kKindLeaf) return (c & 0xFFFF) | (kKindLeaf << 24);
    if (task[c]) return (c & 0xFFFF) | (slot[c] << 16) | (kKindInt << 24);
    const int32_t d0 = desc(c, 0), d1 = desc(c, 1);
    inl[c] = (int)(ient.size() / 4);
    ient.insert(ient.end(), {c, d0, d1, height[c]});
    return (inl[c] & 0xFFFF) | (kKindInline << 24);
  };
  const int n_steps = (int)order.size();
  int32_t* offs = region + 4;
  int32_t* steps = region + lp_steps_offset(ni);
  for (int s = 0; s <= S; ++s) offs[s] = n_steps;
  for (int k = n_steps - 1; k >= 0; --k) offs[stage[order[k]]] = k;
  for (int s = S - 1; s >= 0; --s) offs[s] = std::min(offs[s], offs[s + 1]);
  for (int k = 0; k < n_steps; ++k) {
    const int r = order[k];
    steps[4 * k] = (r & 0xFFFF) | (slot[r] << 16);
    steps[4 * k + 1] = desc(r, 0);
    steps[4 * k + 2] = desc(r, 1);
    steps[4 * k + 3] = r == root ? kStepRoot : 0;
  }
  if (!ient.empty()) std::memcpy(steps + 4LL * n_steps, ient.data(), ient.size() * sizeof(int32_t));
  region[0] = S;
  region[1] = n_slots;
  region[2] = n_steps;
  region[3] = (int)(ient.size() / 4);
  return n_slots;
}

}  // namespace

}  // namespace trex

extern "C" int64_t trex_plan_ints(int B, int n_all) {
  if (B <= 0 || n_all < 2) return 0;
  const int ni = n_all - (n_all + 1) / 2;
  return TREX_PLAN_HEADER_INTS + (int64_t)B * ni * 6 +
         (int64_t)B * (trex::staged_tree_ints(ni) + trex::lp_tree_ints(ni));
}

extern "C" int trex_plan_build(const int32_t* children, int B, int n_all,
                               int32_t* plan, int32_t* info) {
  using namespace trex;
  if (!children || !plan || B <= 0 || n_all < 3 || n_all > 65535)
    return set_error(TREX_E_ARG, "trex_plan_build: bad arguments (B=%d n_all=%d)", B, n_all);
  const int nl = (n_all + 1) / 2;
  const int ni = n_all - nl;
  std::memset(plan, 0, sizeof(int32_t) * TREX_PLAN_HEADER_INTS);
  int32_t* fwd = plan + TREX_PLAN_HEADER_INTS;
  int32_t* bt = fwd + (int64_t)B * ni * 4;
  int32_t* staged = bt + (int64_t)B * ni * 2;
  int32_t* lanes = staged + (int64_t)B * staged_tree_ints(ni);
  int max_slots = 0, all_bt_ok = 1, dag = 0, unr = 0, lp_slots = 0;
  for (int b = 0; b < B; ++b) {
    int s = 0, ok = 0, d = 0, u = 0;
    if (!plan_one_tree(children + (int64_t)b * n_all * 2, n_all, fwd + (int64_t)b * ni * 4,
                       bt + (int64_t)b * ni * 2, &s, &ok, &d, &u))
      return set_error(TREX_E_TOPOLOGY, "trex_plan_build: tree %d has an invalid child list", b);
    stage_one_tree(children + (int64_t)b * n_all * 2, n_all, staged + b * staged_tree_ints(ni));
    const int ls = lane_program_one_tree(children + (int64_t)b * n_all * 2, n_all,
                                         lanes + b * lp_tree_ints(ni));
    lp_slots = (ls < 0 || lp_slots < 0) ? -1 : std::max(lp_slots, ls);
    max_slots = std::max(max_slots, s);
    all_bt_ok &= ok;
    dag += d;
    unr += u;
  }
  plan[0] = kPlanMagic;
  plan[1] = B;
  plan[2] = n_all;
  plan[3] = nl;
  plan[4] = ni;
  plan[5] = max_slots;
  plan[6] = all_bt_ok;
  plan[7] = lp_slots;
  if (info) {
    // low 16 bits: the stack depth; bits 16-23: lane-program slots + 1 (0: a
    // tree of the batch cannot run the lane-per-site kernel)
    info[0] = max_slots | ((lp_slots < 0 ? 0 : lp_slots + 1) << 16);
    info[1] = all_bt_ok;
    info[2] = dag;
    info[3] = unr;
  }
  return TREX_OK;
}

// ---------------------------------------------------------------------------
// Ragged batches: trees of different sizes (n_all_b) and site counts (L_b) in
// one launch.  Layout (ints): header [16] | per-tree records [B][12] |
// work-item -> tree [items] | forward steps [sum n_int_b][4] |
// backtrack entries [sum n_int_b][2].  Record: steps offset, n_int, n_leaves,
// L, first site, first item, leaf byte offset (lo, hi), row-site offset
// (lo, hi), 2 spare.  One work item = one tree x 64-site tile.
// ---------------------------------------------------------------------------
namespace trex {
namespace {
constexpr int32_t kRaggedMagic = 0x54525247;  // 'TRRG'
constexpr int kRaggedMetaInts = 12;           // = kRaggedMeta (sankoff.hip)

bool ragged_shapes(const int32_t* n_all, const int32_t* L, int B, int64_t* steps, int64_t* items) {
  *steps = 0;
  *items = 0;
  for (int b = 0; b < B; ++b) {
    if (n_all[b] < 3 || n_all[b] > 65535 || L[b] <= 0) return false;
    *steps += n_all[b] - (n_all[b] + 1) / 2;
    *items += (L[b] + 63) / 64;
  }
  return *items <= 0x7FFFFFFF;
}
}  // namespace
}  // namespace trex

extern "C" int64_t trex_ragged_plan_ints(int B, const int32_t* n_all, const int32_t* L) {
  if (B <= 0 || !n_all || !L) return 0;
  int64_t steps, items;
  if (!trex::ragged_shapes(n_all, L, B, &steps, &items)) return 0;
  return TREX_PLAN_HEADER_INTS + (int64_t)B * trex::kRaggedMetaInts + items + steps * 6;
}

extern "C" int trex_ragged_plan_build(const int32_t* children, const int32_t* n_all,
                                      const int32_t* L, int B, int32_t* plan, int64_t* info) {
  using namespace trex;
  int64_t steps, items;
  if (!children || !n_all || !L || !plan || B <= 0 || !ragged_shapes(n_all, L, B, &steps, &items))
    return set_error(TREX_E_ARG, "trex_ragged_plan_build: bad arguments (B=%d)", B);
  int32_t* meta = plan + TREX_PLAN_HEADER_INTS;
  int32_t* ritem = meta + (int64_t)B * kRaggedMetaInts;
  int32_t* fwd = ritem + items;
  int32_t* bt = fwd + steps * 4;
  std::memset(plan, 0, sizeof(int32_t) * TREX_PLAN_HEADER_INTS);
  int64_t step_off = 0, item_off = 0, site_off = 0, leaf_off = 0, rows_off = 0, child_off = 0;
  int max_slots = 0, max_nl = 0, max_ni = 0, all_ok = 1, dag = 0, unr = 0;
  for (int b = 0; b < B; ++b) {
    const int na = n_all[b];
    const int nl = (na + 1) / 2;
    const int ni = na - nl;
    int s = 0, ok = 0, d = 0, u = 0;
    if (!plan_one_tree(children + child_off, na, fwd + step_off * 4, bt + step_off * 2, &s, &ok, &d,
                       &u))
      return set_error(TREX_E_TOPOLOGY, "trex_ragged_plan_build: tree %d has an invalid child list",
                       b);
    if (site_off > 0x7FFFFFFF)
      return set_error(TREX_E_UNSUPPORTED, "trex_ragged_plan_build: more than 2^31 sites");
    if ((int64_t)ni * L[b] * 4 * 4 > 0x7FFFFFF0LL)
      return set_error(TREX_E_UNSUPPORTED, "trex_ragged_plan_build: tree %d's DP table exceeds 2 GiB",
                       b);
    int32_t* m = meta + (int64_t)b * kRaggedMetaInts;
    m[0] = (int32_t)step_off;
    m[1] = ni;
    m[2] = nl;
    m[3] = L[b];
    m[4] = (int32_t)site_off;
    m[5] = (int32_t)item_off;
    m[6] = (int32_t)(leaf_off & 0xFFFFFFFF);
    m[7] = (int32_t)(leaf_off >> 32);
    m[8] = (int32_t)(rows_off & 0xFFFFFFFF);
    m[9] = (int32_t)(rows_off >> 32);
    const int tiles = (L[b] + 63) / 64;
    for (int t = 0; t < tiles; ++t) ritem[item_off + t] = b;
    max_slots = std::max(max_slots, s);
    max_nl = std::max(max_nl, nl);
    max_ni = std::max(max_ni, ni);
    all_ok &= ok;
    dag += d;
    unr += u;
    step_off += ni;
    item_off += tiles;
    site_off += L[b];
    leaf_off += (int64_t)nl * L[b];
    rows_off += (int64_t)ni * L[b];
    child_off += 2LL * na;
  }
  plan[0] = kRaggedMagic;
  plan[1] = B;
  plan[2] = (int32_t)steps;
  plan[3] = (int32_t)items;
  plan[4] = max_slots;
  plan[5] = max_nl;
  plan[6] = all_ok;
  plan[7] = max_ni;
  if (info) {
    info[0] = max_slots;  // n_slots for the launch
    info[1] = max_nl;     // LDS leaf tile rows
    info[2] = items;      // work items (64-site tiles)
    info[3] = leaf_off;   // packed leaf bytes: sum n_leaves_b * L_b
    info[4] = rows_off;   // packed DP row-sites: sum n_int_b * L_b (x Q floats)
    info[5] = site_off;   // packed sites: sum L_b
    info[6] = all_ok;     // reference backtrack terminates on every tree
    info[7] = dag + ((int64_t)unr << 32);
  }
  return TREX_OK;
}
