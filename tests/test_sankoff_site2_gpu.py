"""The wave-pair lane-per-site kernel (trex_amd/csrc/sankoff_site2.hip,
TREX_SITE2=1) against the one-wave kernel (sankoff_site.hip) and the fp64
oracle.

The pair kernel splits each site's states over two waves but sums every
mat-vec over all states in the one-wave order, so the DP table, tree and
site scores, marginals and soft ancestral states are bitwise the one-wave
kernel's; dC sums its outer products in another order (16x16 tiles per
wave instead of one 32x32 block) and is checked against the fp64 oracle
at the suite's softmin bar.  Q = 7 leaves the upper wave of every pair
without states (it still joins every pair meeting); 13 and 20 split them.
Every case checks, by the library's launch counter, that the pair kernel
took the calls (TREX_SITE2 names the pair count; the largest whose LDS fits
when "1").
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import (assert_dp_close, assert_grad_close, balanced_children, cond_rtol, int_cost,
                    random_leaves, random_topologies, simulate_leaves)
from oracle.softmin_ref import batched_fwd_bwd_ref
from trex_amd import SankoffEngine, TreePlan, children_from_adjacency
from trex_amd._lib import lib

pytestmark = pytest.mark.gpu


def _dev(x, device, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(device).contiguous()


def _runs(monkeypatch, ch, leaves, cost, L, Q, tau, device, hard_root=False, dts=None,
          pairs="1"):
    lv, c = _dev(leaves, device), _dev(cost, device, torch.float32)
    kw = dict(hard_root=hard_root)
    out = []
    for flag in (pairs, "0"):
        monkeypatch.setenv("TREX_SITE2", flag)
        n0 = lib().trex_debug_site2_launches()
        eng = SankoffEngine(TreePlan(ch), L, Q, device)
        f, dc, mg, an = eng.fwd_bwd(lv, c, tau, dts, site_score=True, marginals=True,
                                    anc_states=True, **kw)
        f2 = eng.forward(lv, c, tau, site_score=True, **kw)
        dc2, mg2, an2 = eng.backward(lv, c, tau, f2.dp, dts, marginals=True, anc_states=True, **kw)
        torch.cuda.synchronize()
        # the wave-pair kernel took exactly the three calls (fused, forward, adjoint)
        assert lib().trex_debug_site2_launches() - n0 == (3 if flag != "0" else 0), flag
        out.append(dict(dp=f.dp.clone(), tree=f.tree_score.clone(), site=f.site_score.clone(),
                        dc=dc.clone(), marg=mg.clone(), anc=an.clone(), dp2=f2.dp.clone(),
                        tree2=f2.tree_score.clone(), site2=f2.site_score.clone(), dc2=dc2.clone(),
                        marg2=mg2.clone(), anc2=an2.clone()))
    return out


@pytest.mark.parametrize("pairs", ["8", "6", "4"])
@pytest.mark.parametrize("topo", ["balanced", "random"])
@pytest.mark.parametrize("Q", [20, 13, 7])
def test_site2_matches_site_kernel(device, monkeypatch, topo, Q, pairs):
    B, n, L, tau = 2, 48, 777, 0.5  # 48 taxa: every pair count's LDS fits
    ch = balanced_children(n, B) if topo == "balanced" else random_topologies(B, n, seed=91)
    leaves = random_leaves(B, n, L, Q, seed=92, missing=0.03)
    cost = int_cost(Q, seed=93)
    pair, one = _runs(monkeypatch, ch, leaves, cost, L, Q, tau, device, pairs=pairs)
    for k in ("dp", "tree", "site", "marg", "anc", "dp2", "tree2", "site2", "marg2", "anc2"):
        assert torch.equal(pair[k], one[k]), k
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    rt = cond_rtol(ref["dp"], tau)
    assert_grad_close(pair["dc"].cpu().numpy(), ref["d_cost"], rtol=rt)
    assert_grad_close(pair["dc2"].cpu().numpy(), ref["d_cost"], rtol=rt)
    np.testing.assert_allclose(pair["dc"].cpu().numpy(), one["dc"].cpu().numpy(), rtol=1e-5,
                               atol=1e-6 * float(one["dc"].abs().max()))


def test_site2_hard_root_and_tree_cotangents(device, monkeypatch):
    """The root's hard minimum (wave 0 of the workgroup scores the site from
    both halves' D) and per-tree score cotangents: bitwise the one-wave
    kernel for everything but dC, dC vs the one-wave kernel's."""
    B, n, L, Q, tau = 3, 40, 300, 20, 0.5
    ch = random_topologies(B, n, seed=95)
    leaves = random_leaves(B, n, L, Q, seed=96, missing=0.05)
    cost = int_cost(Q, seed=97)
    dts = torch.tensor([1.0, -0.5, 2.0], device=device)
    pair, one = _runs(monkeypatch, ch, leaves, cost, L, Q, tau, device, hard_root=True, dts=dts)
    for k in ("dp", "tree", "site", "marg", "anc", "dp2", "marg2", "anc2"):
        assert torch.equal(pair[k], one[k]), k
    for k in ("dc", "dc2"):
        np.testing.assert_allclose(pair[k].cpu().numpy(), one[k].cpu().numpy(), rtol=1e-5,
                                   atol=1e-6 * float(one[k].abs().max()))


def test_site2_c3_scale(device, monkeypatch):
    """BASELINE C3's size (64 taxa x 10 000 sites x 20 states, tau 0.5):
    bitwise the one-wave kernel, dC at the suite's bar vs the fp64 oracle."""
    n, L, Q, tau = 64, 10000, 20, 0.5
    # the bench's C3 tree (bench.py / tools/time_small.py: 12 lane-program
    # slots, so the one-wave kernel takes it too)
    seqs, adj = simulate_leaves(n, L, Q, 50, seed=2)
    ch = children_from_adjacency(adj)
    leaves = np.ascontiguousarray(seqs[None, :n])
    cost = int_cost(Q, seed=3)
    pair, one = _runs(monkeypatch, ch, leaves, cost, L, Q, tau, device)
    for k in ("dp", "tree", "site", "marg", "anc", "dp2", "marg2", "anc2"):
        assert torch.equal(pair[k], one[k]), k
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    assert_grad_close(pair["dc"].cpu().numpy(), ref["d_cost"], rtol=1e-5)
    assert_dp_close(pair["dp"].cpu().numpy().transpose(0, 1, 3, 2), ref, 1e-5)
