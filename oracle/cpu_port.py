"""ctypes wrapper of oracle/libsankoff_cpu.so (OpenMP C restatement).

TEST INFRASTRUCTURE / CPU BASELINE ONLY -- see oracle/cpu_port.c.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libsankoff_cpu.so")
        if not os.path.exists(path):
            import subprocess

            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        _LIB = ctypes.CDLL(path)
        p = ctypes.c_void_p
        i = ctypes.c_int
        for fn in (_LIB.sankoff_cpu_fwd_bwd, _LIB.sankoff_cpu64_fwd_bwd):
            fn.restype = i
            fn.argtypes = [p, p, p, i, i, i, i, ctypes.c_float, p, p, p, i, i]
    return _LIB


def fwd_bwd(children, leaves, cost, tau, want_dp=False, want_grad=True, threads=0,
            precision="f32"):
    """Returns (tree_score (B,) f64, d_cost (Q,Q) f64, dp (B,n_int,Q,L) f32 | None).

    precision "f32": trex's fp32 arithmetic (the timed CPU baseline);
    "f64": the same recurrence in fp64 (the checker for full-batch GPU runs,
    pinned to oracle/softmin_ref by tests/test_cpu_port_cpu.py)."""
    if precision not in ("f32", "f64"):
        raise ValueError(precision)
    ch = np.ascontiguousarray(children, dtype=np.int32)
    lv = np.ascontiguousarray(leaves, dtype=np.int8)
    c = np.ascontiguousarray(cost, dtype=np.float32)
    B, n_all, _ = ch.shape
    L = lv.shape[2]
    Q = c.shape[0]
    nl = (n_all + 1) // 2
    dp = np.empty((B, n_all - nl, Q, L), np.float32) if want_dp else None
    ts = np.zeros(B, np.float64)
    dc = np.zeros((Q, Q), np.float64)
    fn = _lib().sankoff_cpu_fwd_bwd if precision == "f32" else _lib().sankoff_cpu64_fwd_bwd
    rc = fn(ch.ctypes.data, lv.ctypes.data, c.ctypes.data, B, L, n_all,
            Q, float(tau), None if dp is None else dp.ctypes.data, ts.ctypes.data,
            dc.ctypes.data, 1 if want_grad else 0, int(threads))
    if rc != 0:
        raise ValueError("sankoff_cpu_fwd_bwd: bad arguments")
    return ts, dc, dp
