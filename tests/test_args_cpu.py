"""C-ABI argument validation, callable without a GPU.

The library is compiled with -fno-honor-nans (the kernels drop NaN
canonicalisation), so its host-side float checks test the IEEE bit pattern
instead of comparisons the compiler may fold.  Every call below
is rejected before any launch, so it runs on the CPU container: host numpy
buffers stand in for device pointers and are never touched.
"""

from __future__ import annotations

import numpy as np
import pytest

from trex_amd._lib import TREX_E_ARG, lib


def _buf(n=1 << 16):
    return np.zeros(n, np.uint8)


BAD = [float("nan"), float("inf"), -float("inf"), -1.0, -1e-30]


@pytest.mark.parametrize("tau", BAD)
def test_sankoff_rejects_bad_tau(tau):
    b = _buf()
    p = b.ctypes.data
    L = lib()
    ws = int(L.trex_workspace_bytes(1, 64, 7, 4))
    w = _buf(ws)
    rc = L.trex_sankoff_fwd(p, 2, p, p, 1, 64, 7, 4, tau, 0, p, None, p, w.ctypes.data, ws, None)
    assert rc == TREX_E_ARG, (tau, rc)
    assert b"tau" in L.trex_last_error()
    rc = L.trex_sankoff_fwd_bwd(p, 2, p, p, 1, 64, 7, 4, tau, 0, p, None, p, None, p, None, None,
                                w.ctypes.data, ws, None)
    assert rc == TREX_E_ARG


@pytest.mark.parametrize("Q", [4, 20])
@pytest.mark.parametrize("flags", [2, 4, 0x80000000])
def test_sankoff_rejects_unknown_flags(Q, flags):
    """v9: only TREX_FLAG_HARD_ROOT is a flag (v8's TREX_FLAG_SITE_REUSE = 2
    is refused, not silently ignored)."""
    b = _buf()
    p = b.ctypes.data
    L = lib()
    ws = int(L.trex_workspace_bytes(1, 64, 7, Q))
    w = _buf(ws)
    rc = L.trex_sankoff_fwd(p, 2, p, p, 1, 64, 7, Q, 0.5, flags, p, None, p, w.ctypes.data, ws,
                            None)
    assert rc == TREX_E_ARG, (flags, rc)
    assert b"flags" in L.trex_last_error()


@pytest.mark.parametrize("bad", [float("nan"), float("inf"), 0.0, -2.0])
def test_split_gemms_reject_bad_bounds(bad):
    b = _buf()
    p = b.ctypes.data
    L = lib()
    ws = int(L.trex_tree_workspace_bytes(64, 256))
    w = _buf(ws)
    assert L.trex_tree_gram_skip_x3(p, 64, 256, 0, bad, p, w.ctypes.data, ws, None) == TREX_E_ARG
    assert L.trex_tree_mf_rows_x3(p, p, 64, 256, 0, 64, bad, 1.0, p, None) == TREX_E_ARG
    assert L.trex_tree_mf_rows_x3(p, p, 64, 256, 0, 64, 65.0, bad, p, None) == TREX_E_ARG


@pytest.mark.parametrize("bad", [float("nan"), float("inf"), 0.0, -1.0])
def test_temperatures_reject_bad_values(bad):
    b = _buf()
    p = b.ctypes.data
    L = lib()
    assert L.trex_tree_update_tree(p, None, None, 7, 3, bad, p, None) == TREX_E_ARG
    assert L.trex_tree_update_tree_bwd(p, p, None, 7, 3, bad, p, None) == TREX_E_ARG


@pytest.mark.parametrize("Q,short", [(5, False), (2, False), (4, True)])
def test_leaf_code_mf_rejects_wrong_alphabet_or_short_buffer(Q, short):
    """trex_tree_mf_rows_x3_codes reads one code byte per (code row, site) of
    a Q = 4 alphabet: any other Q, or a codes buffer smaller than
    trex_tree_leaf_codes_bytes(n_leaf, K / Q), is TREX_E_ARG."""
    b = _buf()
    p = b.ctypes.data
    L = lib()
    N, n_leaf, sites = 127, 64, 100
    K = sites * Q
    need = int(L.trex_tree_leaf_codes_bytes(n_leaf, sites))
    rc = L.trex_tree_mf_rows_x3_codes(p, p, N, K, n_leaf, N - n_leaf, 128.0, 1.0, p,
                                      need - 1 if short else need, n_leaf, Q, p, None)
    assert rc == TREX_E_ARG, rc
    assert b"codes" in L.trex_last_error()


@pytest.mark.parametrize("bad", [float("nan"), float("inf"), 0.0, -2.0])
def test_presplit_and_fused_step_entries_reject_bad_args(bad):
    """The x3p (pre-split operand) entry points and the fused C5 step entry
    points reject bad bounds / temperatures / shapes before any launch."""
    b = _buf()
    p = b.ctypes.data
    L = lib()
    ws = int(L.trex_tree_workspace_bytes(64, 256))
    w = _buf(ws)
    assert L.trex_tree_split_x3(p, 64, 256, 256, bad, p, 256, None) == TREX_E_ARG
    assert L.trex_tree_split_x3(p, 64, 256, 256, 1.0, p, 254, None) == TREX_E_ARG  # ldo % 4
    assert L.trex_tree_gram_skip_x3p(p, 64, 256, 0, bad, p, w.ctypes.data, ws, None) == TREX_E_ARG
    assert L.trex_tree_gram_skip_x3p_codes(p, 64, 256, 0, bad, p, 4096, 32, 4, p, w.ctypes.data,
                                           ws, None) == TREX_E_ARG
    assert L.trex_tree_gram_skip_x3p_codes(p, 64, 256, 0, 1.0, None, 4096, 32, 4, p,
                                           w.ctypes.data, ws, None) == TREX_E_ARG  # no codes
    assert L.trex_tree_gram_skip_x3p_codes(p, 64, 256, 0, 1.0, p, 4096, 32, 5, p, w.ctypes.data,
                                           ws, None) == TREX_E_ARG  # Q = 4 only
    assert L.trex_tree_gram_skip_x3p_codes(p, 64, 256, 0, 1.0, p, 100, 32, 4, p, w.ctypes.data,
                                           ws, None) == TREX_E_ARG  # codes buffer too small
    assert L.trex_tree_mf_rows_x3p(p, 64, p, 64, 256, 0, 64, bad, 1.0, None, 0, 32, 4, p,
                                   None) == TREX_E_ARG
    assert L.trex_tree_mf_rows_x3p(p, 64, p, 64, 258, 0, 64, 65.0, 1.0, None, 0, 32, 4, p,
                                   None) == TREX_E_ARG  # K % 4
    assert L.trex_adam_seq_update_step_x3p(p, 8, 16, 4, bad, 1.0, p, p, p, 1, 0.01, 0.9, 0.999,
                                           1e-8, None, 1.0, p, None) == TREX_E_ARG
    assert L.trex_adam_seq_update_step_x3p(p, 8, 16, 5, 1.0, 1.0, p, p, p, 1, 0.01, 0.9, 0.999,
                                           1e-8, None, 1.0, p, None) == TREX_E_ARG  # Q = 4 only
    assert L.trex_tree_update_tree_bwd_adam(p, p, None, 7, 3, bad, p, p, p, p, 1, None, 0.01,
                                            0.9, 0.999, 1e-8, None) == TREX_E_ARG
    assert L.trex_tree_update_tree_bwd_adam(p, p, None, 7, 3, 1.0, p, p, p, p, 0, None, 0.01,
                                            0.9, 0.999, 1e-8, None) == TREX_E_ARG  # count 0
    assert L.trex_tree_surrogate_constraint(p, p, 7, 10.0, 1.0, None, p, p, p, 8.0, p, 6,
                                            w.ctypes.data, None) == TREX_E_ARG  # ldm16 < N
