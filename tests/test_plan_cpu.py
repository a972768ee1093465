"""CPU tests of the host side of libtrexhip.so: exports, the topology planner
(checked by executing its program with a numpy interpreter), adjacency
conversion.  No kernel is launched here."""

from __future__ import annotations

import ctypes
import os
import re

import numpy as np
import pytest

from _cases import balanced_children, int_cost, random_leaves, random_topologies, weird_children
from oracle.sankoff_ref import SENTINEL, leaf_dp, trex_children_table
from oracle.softmin_ref import batched_fwd_bwd_ref
from trex_amd import TreePlan, children_from_adjacency, create_balanced_binary_tree, lib
from trex_amd._lib import SIGNATURES
from trex_amd.topology import adjacency_from_children

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    with open(os.path.join(ROOT, "include", "trex_hip.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(trex_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    handle = ctypes.CDLL(str(lib()._name))
    names = _header_functions()
    assert len(names) >= 9
    for n in names:
        assert hasattr(handle, n), n
        assert n in SIGNATURES, f"{n} missing from trex_amd._lib.SIGNATURES"


def test_children_from_adjacency_matches_trex_rule():
    adj = create_balanced_binary_tree(16)
    adj[-1, -1] = 1  # root self loop is removed by run_sankoff (sankoff.py:141)
    ch = children_from_adjacency(adj)[0]
    np.testing.assert_array_equal(ch, trex_children_table(adj))
    rng = np.random.default_rng(0)
    for _ in range(5):
        a = (rng.random((9, 9)) < 0.3).astype(np.float32)
        a[rng.random((9, 9)) < 0.1] = 0.5  # non-1 values are not edges (== 1 test)
        np.testing.assert_array_equal(children_from_adjacency(a)[0], trex_children_table(a))


def _interpret(plan: TreePlan, b, leaves, cost):
    """Execute the encoded forward program with an explicit slot stack."""
    steps = plan.fwd_steps[b]
    Q = cost.shape[0]
    L = leaves.shape[-1]
    slots = {}
    dp = np.full((plan.n_int, L, Q), np.nan)
    lD = leaf_dp(leaves, Q)
    last = None
    prev, prev_row = None, -1
    for row_desc, da, db, flags in steps:
        row = row_desc & 0xFFFF
        oslot = (row_desc >> 16) & 0xFF
        acc = np.zeros((L, Q))
        for d in (da, db):
            kind = (d >> 24) & 3
            if kind == 1:
                D = lD[d & 0xFFFF]
            elif kind == 2 and d & (1 << 27):  # register bypass: previous step's output
                assert prev_row == d & 0xFFFF, "bypass child is not the previous step"
                D = prev
            elif kind == 2:
                s = (d >> 16) & 0xFF
                D = slots[s]
                assert np.array_equal(D, dp[d & 0xFFFF]), "slot clobbered"
            else:
                D = np.full((L, Q), SENTINEL)
            acc = acc + (cost[None] + D[:, None, :]).min(axis=2)
        dp[row] = acc
        if oslot != 0xFF and not flags & 4:
            slots[oslot] = acc
        prev, prev_row = acc, row
        last = row
    assert last == plan.n_int - 1, "root must be the last step"
    return dp


@pytest.mark.parametrize("kind", ["random", "balanced", "fwdref", "dag", "cycle"])
def test_plan_program_reproduces_oracle(kind):
    if kind == "random":
        ch = random_topologies(4, 40, seed=1)
    elif kind == "balanced":
        ch = balanced_children(64, B=2)
    else:
        ch = weird_children(kind)[None]
    plan = TreePlan(ch)
    n_all = ch.shape[1]
    nl = (n_all + 1) // 2
    leaves = random_leaves(ch.shape[0], nl, 11, 4, seed=2, missing=0.1)
    cost = int_cost(4, seed=3)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, 0.0)
    for b in range(ch.shape[0]):
        dp = _interpret(plan, b, leaves[b], cost.astype(np.float64))
        np.testing.assert_array_equal(dp.transpose(0, 2, 1), ref["dp"][b])
    assert plan.backtrack_ok == (0 if kind == "cycle" else 1)


@pytest.mark.parametrize("kind", ["random", "balanced", "fwdref", "dag", "cycle", "unreached"])
def test_plan_deferred_cherries(kind):
    """kChildDeferred (bit 28 of a child descriptor) / kStepDeferredIn (flag
    8, trex_common.h): exactly the cherries (both children leaves or
    sentinels) with one reached parent are deferred, each by its one parent,
    and every deferred cherry is stepped before its parent (its adjoint step
    comes after the parent's, which hands it the parent's cotangent)."""
    if kind == "random":
        ch = random_topologies(4, 40, seed=1)
    elif kind == "balanced":
        ch = balanced_children(64, B=2)
    elif kind == "unreached":
        # 13 becomes an orphan: its cherry 11 has one (unreached) parent,
        # cherry 10 two parents (14, 13)
        ch = balanced_children(8).copy()
        ch[0, 14] = (12, 10)
    else:
        ch = weird_children(kind)[None]
    plan = TreePlan(ch)
    nl = (ch.shape[1] + 1) // 2
    ni = ch.shape[1] - nl
    n_def = 0
    for b in range(ch.shape[0]):
        steps = [tuple(int(x) for x in s) for s in plan.fwd_steps[b]]
        pos = {s[0] & 0xFFFF: k for k, s in enumerate(steps)}
        flags = {s[0] & 0xFFFF: s[3] for s in steps}
        kids = {s[0] & 0xFFFF: (s[1], s[2]) for s in steps}
        parents = {}
        for s in steps:
            for d in (s[1], s[2]):
                if (d >> 24) & 3 == 2:
                    parents.setdefault(d & 0xFFFF, []).append((s[0] & 0xFFFF, d))
        for r in range(ni):
            cherry = all((d >> 24) & 3 != 2 for d in kids[r])
            ps = parents.get(r, [])
            want = cherry and len(ps) == 1 and not flags[ps[0][0]] & 2
            assert bool(flags[r] & 8) == want, (b, r)
            for p, d in ps:
                assert bool(d & (1 << 28)) == want
                if want:
                    assert pos[r] < pos[p] and not d & (1 << 26)
            n_def += want
    if kind in ("random", "balanced"):
        assert n_def > 0


STAGE_WAVES = 8  # kStageWaves (trex_common.h)


def _staged(plan, b):
    """Decode tree b's staged region (trex_common.h): steps, S, offsets."""
    from trex_amd._lib import TREX_PLAN_HEADER_INTS

    ni, W = plan.n_int, STAGE_WAVES
    stride = 4 * ni + ((ni * W + 2 + 3) & ~3)
    base = TREX_PLAN_HEADER_INTS + plan.B * ni * 6 + b * stride
    r = plan.host[base:base + stride]
    S = int(r[4 * ni])
    return r[:4 * ni].reshape(ni, 4), S, r[4 * ni + 1:4 * ni + 2 + S * W]


@pytest.mark.parametrize("kind", ["random", "balanced", "fwdref", "dag", "cycle"])
def test_staged_program_reproduces_oracle(kind):
    """The staged (multi-wave) program of sankoff_staged.hip: run with the
    waves of every stage in reverse order (any interleaving must do), it
    reproduces the oracle DP table; in the adjoint order no two waves of a
    stage write one cotangent slot, every slot is set before it is
    accumulated into or read, and the DAG quirk runs serially on wave 0."""
    if kind == "random":
        ch = random_topologies(4, 40, seed=1)
    elif kind == "balanced":
        ch = balanced_children(64, B=2)
    else:
        ch = weird_children(kind)[None]
    plan = TreePlan(ch)
    n_all = ch.shape[1]
    nl = (n_all + 1) // 2
    ni = n_all - nl
    W = STAGE_WAVES
    leaves = random_leaves(ch.shape[0], nl, 11, 4, seed=2, missing=0.1)
    cost = int_cost(4, seed=3).astype(np.float64)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, 0.0)
    for b in range(ch.shape[0]):
        steps, S, offs = _staged(plan, b)
        assert np.all(np.diff(offs) >= 0) and offs[0] == 0 and offs[-1] == ni
        assert sorted(steps[:, 0] & 0xFFFF) == list(range(ni))
        stage_of = {}
        for s in range(S):
            for w in range(W):
                for k in range(offs[s * W + w], offs[s * W + w + 1]):
                    stage_of[int(steps[k, 0] & 0xFFFF)] = (s, w, k)
        if plan.n_dag_nodes:
            assert S == 1 and all(v[1] == 0 for v in stage_of.values())
        lD = leaf_dp(leaves[b], 4)
        dp = np.full((ni, 11, 4), np.nan)
        for s in range(S):
            for w in reversed(range(W)):
                for k in range(offs[s * W + w], offs[s * W + w + 1]):
                    row, da, db, flags = (int(x) for x in steps[k])
                    acc = np.zeros((11, 4))
                    for d in (da, db):
                        kind_ = (d >> 24) & 3
                        if kind_ == 1:
                            D = lD[d & 0xFFFF]
                        elif kind_ == 2:
                            D = dp[d & 0xFFFF]
                            assert not np.isnan(D).any(), "child not computed in an earlier stage"
                            cs = stage_of[d & 0xFFFF]
                            assert cs[0] < s or (cs[1] == w and cs[2] < k)
                        else:
                            D = np.full((11, 4), SENTINEL)
                        acc = acc + (cost[None] + D[:, None, :]).min(axis=2)
                    dp[row & 0xFFFF] = acc
        np.testing.assert_array_equal(dp.transpose(0, 2, 1), ref["dp"][b])
        # adjoint: stages and each wave's steps reversed
        state = {ni - 1: "set"}
        for s in reversed(range(S)):
            writers = {}
            for w in range(W):
                for k in reversed(range(offs[s * W + w], offs[s * W + w + 1])):
                    row, da, db, flags = (int(x) for x in steps[k])
                    if flags & 2:  # unreached
                        continue
                    assert state.get(row & 0xFFFF) == "set", "cotangent read before it is set"
                    for d in (da, db):
                        if (d >> 24) & 3 != 2:
                            continue
                        c = d & 0xFFFF
                        assert writers.setdefault(c, w) == w, "two waves write one slot in a stage"
                        if d & (1 << 26):
                            assert state.get(c) == "set", "accumulate into an unset slot"
                        else:
                            assert c not in state, "slot set twice"
                        state[c] = "set"


def test_plan_slot_counts_are_sethi_ullman():
    """Sethi-Ullman depth minus the register bypass: the child evaluated
    right before its parent never takes a slot, so a balanced tree of n
    leaves needs log2(n) slots (not log2(n) + 1) and a caterpillar none."""
    for n, want in [(8, 2), (64, 5), (256, 7)]:
        assert TreePlan.from_adjacency(create_balanced_binary_tree(n)).n_slots == want
    # a caterpillar: every internal child is the previous step
    n = 20
    ch = np.full((1, 2 * n - 1, 2), -1, np.int32)
    ch[0, n] = (0, 1)
    for k in range(1, n - 1):
        ch[0, n + k] = (k + 1, n + k - 1)
    assert TreePlan(ch).n_slots == 0


def test_plan_rejects_bad_children():
    from trex_amd import TrexError

    ch = balanced_children(8)
    ch[0, 9, 0] = 99
    with pytest.raises(TrexError):
        TreePlan(ch)


def test_adjacency_roundtrip():
    ch = random_topologies(3, 12, seed=5)
    np.testing.assert_array_equal(children_from_adjacency(adjacency_from_children(ch)), ch)


def test_abi_version_matches_plan_layout():
    """trex_version() >= 6: plans carry the lane-per-site program of every
    tree after the staged programs, and info[0] packs its slot count above
    the stack depth (include/trex_hip.h); a binding that sized v5 plans
    itself must see the bump.  7 added the device step state (no plan
    change)."""
    assert lib().trex_version() == 10
    ch = balanced_children(64, B=1)
    p = TreePlan(ch)
    assert p.n_slots == 5 and p.lane_slots == 12 and p.slot_word == 5 | (13 << 16)


def _lanes(plan, b):
    """Decode tree b's lane-per-site region (trex_common.h)."""
    from trex_amd._lib import TREX_PLAN_HEADER_INTS

    ni, W = plan.n_int, STAGE_WAVES
    staged = 4 * ni + ((ni * W + 2 + 3) & ~3)
    steps_off = 8 + ((ni + 1 + 3) & ~3)
    stride = steps_off + 4 * ni
    base = TREX_PLAN_HEADER_INTS + plan.B * ni * 6 + plan.B * staged + b * stride
    r = plan.host[base:base + stride]
    S, n_slots, n_steps, n_inl = (int(x) for x in r[:4])
    offs = r[4:5 + S]
    steps = r[steps_off:steps_off + 4 * n_steps].reshape(n_steps, 4)
    inl = r[steps_off + 4 * n_steps:steps_off + 4 * (n_steps + n_inl)].reshape(n_inl, 4)
    return S, n_slots, offs, steps, inl


@pytest.mark.parametrize("kind", ["random", "balanced", "fwdref", "dag", "cycle", "small"])
def test_lane_program_reproduces_oracle(kind):
    """The lane-per-site program of sankoff_site.hip, executed stage by stage
    with an LDS-slot model: every internal row is computed exactly once
    (task or inline), a task's task children finish in earlier stages, no
    slot is overwritten while live (forward D, then adjoint cotangent over
    the same interval), and the D of every row equals the oracle DP table.
    Trees with a shared child or an unreached row have no program."""
    if kind == "random":
        ch = random_topologies(4, 40, seed=1)
    elif kind == "balanced":
        ch = balanced_children(64, B=2)
    elif kind == "small":
        ch = balanced_children(2, B=1)
    else:
        ch = weird_children(kind)[None]
    plan = TreePlan(ch)
    n_all = ch.shape[1]
    nl = (n_all + 1) // 2
    ni = n_all - nl
    L, Q = 11, 4
    leaves = random_leaves(ch.shape[0], nl, L, Q, seed=2, missing=0.1)
    cost = int_cost(Q, seed=3).astype(np.float64)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, 0.0)
    for b in range(ch.shape[0]):
        S, n_slots, offs, steps, inl = _lanes(plan, b)
        if n_slots < 0:
            assert plan.n_dag_nodes or plan.n_unreached or kind in ("dag", "cycle", "fwdref")
            assert plan.lane_slots == -1
            continue
        lD = leaf_dp(leaves[b], Q)
        dp = np.full((ni, L, Q), np.nan)
        slot_val = {}   # slot -> row currently held
        done = set()

        def msg(D):
            return (cost[None] + D[:, None, :]).min(axis=2)

        def leafish(d):
            k = (d >> 24) & 3
            assert k in (0, 1)
            return lD[d & 0xFFFF] if k == 1 else np.full((L, Q), SENTINEL)

        def inline_d(idx, depth=0):
            row, da, db, h = (int(x) for x in inl[idx])
            acc = 0
            for d in (da, db):
                if (d >> 24) & 3 == 3:
                    assert depth == 0 and h == 2
                    acc = acc + msg(inline_d(d & 0xFFFF, 1))
                else:
                    acc = acc + msg(leafish(d))
            dp[row] = acc
            done.add(row)
            return dp[row]

        for s in range(S):
            # the stage's tasks run on different waves at once: the slots it
            # writes (its rows') and reads (task children's) are disjoint
            fw = [(int(steps[k][0]) >> 16) & 0xFF for k in range(offs[s], offs[s + 1])]
            fr = {(int(d) >> 16) & 0xFF for k in range(offs[s], offs[s + 1])
                  for d in steps[k][1:3] if (int(d) >> 24) & 3 == 2}
            assert not fr & set(fw) and len(fw) == len(set(fw))
            for k in range(offs[s], offs[s + 1]):
                w0, da, db, flags = (int(x) for x in steps[k])
                row, sl = w0 & 0xFFFF, (w0 >> 16) & 0xFF
                acc = 0
                for d in (da, db):
                    kd = (d >> 24) & 3
                    if kd == 2:
                        c, cs = d & 0xFFFF, (d >> 16) & 0xFF
                        assert slot_val.get(cs) == c, "task child not in its slot"
                        acc = acc + msg(dp[c])
                    elif kd == 3:
                        acc = acc + msg(inline_d(d & 0xFFFF))
                    else:
                        acc = acc + msg(leafish(d))
                dp[row] = acc
                assert row not in done
                done.add(row)
                if flags & 1:
                    assert row == ni - 1 and s == S - 1 and offs[s + 1] - offs[s] == 1
                assert 0 <= sl < n_slots
                slot_val[sl] = row  # overwrites only dead rows (checked by the reads above)
        assert done == set(range(ni))
        np.testing.assert_array_equal(dp.transpose(0, 2, 1), ref["dp"][b])
        # adjoint: the same intervals in reverse -- a task's cotangent is written
        # into its slot at its parent's stage and read at its own stage
        holder = {}
        for s in reversed(range(S)):
            # a stage's tasks (and, at <= 4 tasks, a task's two children) run
            # on different waves at once: no slot written in the stage may be
            # one read in it, and no two writes may share a slot
            reads = {(int(steps[k][0]) >> 16) & 0xFF for k in range(offs[s], offs[s + 1])}
            writes = [(int(d) >> 16) & 0xFF for k in range(offs[s], offs[s + 1])
                      for d in steps[k][1:3] if (int(d) >> 24) & 3 == 2]
            assert not reads & set(writes) and len(writes) == len(set(writes))
            for k in range(offs[s], offs[s + 1]):
                w0, da, db, flags = (int(x) for x in steps[k])
                row, sl = w0 & 0xFFFF, (w0 >> 16) & 0xFF
                if flags & 1:
                    holder[sl] = row  # the root's cotangent, written at the adjoint's start
                assert holder.get(sl) == row, "cotangent slot overwritten before its read"
                for d in (da, db):
                    if (d >> 24) & 3 == 2:
                        holder[(d >> 16) & 0xFF] = d & 0xFFFF
    if kind == "balanced":
        assert plan.lane_slots == 12
