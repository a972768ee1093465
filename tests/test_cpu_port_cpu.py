"""Pins oracle/cpu_port.c (the OpenMP C restatement) to the numpy fp64 oracle.

The fp64 instantiation (`precision="f64"`) is the checker the GPU tests use
where the numpy oracle cannot hold the batch (C4's 1 024 trees,
tests/test_configs_full_gpu.py); the fp32 one is the timed CPU baseline.
Neither may drift from oracle/softmin_ref.py, which restates
src/trex/sankoff.py:24-94,187 (hard) and the build-defined softmin.
"""

from __future__ import annotations

import numpy as np
import pytest

from _cases import (assert_grad_close, hamming, int_cost, random_leaves, random_topologies,
                    weird_children)
from oracle import cpu_port
from oracle.softmin_ref import batched_fwd_bwd_ref


def _case(kind, Q):
    if kind == "random":
        B, n, L = 5, 24, 333
        ch = random_topologies(B, n, seed=7 + Q)
        lv = random_leaves(B, n, L, Q, seed=8 + Q)
    elif kind == "missing":
        B, n, L = 3, 16, 200
        ch = random_topologies(B, n, seed=9)
        lv = random_leaves(B, n, L, Q, seed=10, missing=0.03)
    else:  # trex child quirks: -1 fills, forward references, shared children
        ch = np.stack([weird_children("fwdref"), weird_children("dag")])
        lv = random_leaves(2, 8, 130, Q, seed=11)
    return ch, lv


@pytest.mark.parametrize("kind", ["random", "missing", "quirks"])
@pytest.mark.parametrize("Q", [4, 20])
@pytest.mark.parametrize("tau", [0.0, 0.5, 0.1])
def test_cpu_port_f64_equals_numpy_oracle(kind, Q, tau):
    """fp64 port == fp64 oracle to accumulation-order rounding (1e-11)."""
    ch, lv = _case(kind, Q)
    cost = hamming(Q) if Q == 4 else int_cost(Q, seed=3)
    tau32 = float(np.float32(tau))  # the port takes tau as fp32, like the kernels
    ref = batched_fwd_bwd_ref(ch, lv, cost, tau32)
    ts, dc, dp = cpu_port.fwd_bwd(ch, lv, cost, tau32, want_dp=True, precision="f64")
    np.testing.assert_allclose(ts, ref["tree_score"], rtol=1e-11)
    assert_grad_close(dc, ref["d_cost"], rtol=1e-11)
    np.testing.assert_allclose(dp, ref["dp"].astype(np.float32), rtol=1e-6, atol=1e-9)
    if tau == 0.0:
        assert np.array_equal(ts, ref["tree_score"])
        assert np.array_equal(dp, ref["dp"].astype(np.float32))


@pytest.mark.parametrize("tau", [0.0, 0.5])
def test_cpu_port_f32_baseline_tracks_oracle(tau):
    """The fp32 baseline computes what trex computes: hard scores exact
    (integer values < 2^24), softmin within fp32 rounding of the fp64 oracle."""
    ch, lv = _case("random", 4)
    cost = hamming(4)
    ref = batched_fwd_bwd_ref(ch, lv, cost, tau)
    ts, dc, _ = cpu_port.fwd_bwd(ch, lv, cost, tau, precision="f32")
    if tau == 0.0:
        assert np.array_equal(ts, ref["tree_score"])
        np.testing.assert_allclose(dc, ref["d_cost"], rtol=1e-6)
    else:
        np.testing.assert_allclose(ts, ref["tree_score"], rtol=1e-5)
        assert_grad_close(dc, ref["d_cost"], rtol=1e-4)


def test_cpu_port_rejects_bad_arguments():
    with pytest.raises(ValueError):
        cpu_port.fwd_bwd(np.zeros((1, 3, 2), np.int32), np.zeros((1, 2, 4), np.int8),
                         hamming(40), 0.5)
    with pytest.raises(ValueError):
        cpu_port.fwd_bwd(np.zeros((1, 3, 2), np.int32), np.zeros((1, 2, 4), np.int8),
                         hamming(4), 0.5, precision="bf16")
