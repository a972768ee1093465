"""ctypes binding of libtrexhip.so (C ABI declared in include/trex_hip.h).

The product path has no CPU fallback: if the shared library is missing or a
call fails, this module raises.  Build it with ``python -c "import
__graft_entry__ as g; g.build()"`` (or ``make -C trex_amd/csrc``).
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("TREX_HIP_LIB", _HERE / "libtrexhip.so"))

TREX_OK = 0
TREX_E_ARG = -1
TREX_E_TOPOLOGY = -2
TREX_E_UNSUPPORTED = -3
TREX_E_HIP = -4
TREX_FLAG_HARD_ROOT = 1
TREX_PLAN_HEADER_INTS = 16

_c_i = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_f = ctypes.c_float
_c_u = ctypes.c_uint
_p = ctypes.c_void_p

# name -> (restype, argtypes); must match include/trex_hip.h
SIGNATURES = {
    "trex_last_error": (ctypes.c_char_p, []),
    "trex_version": (_c_i, []),
    "trex_plan_ints": (_c_i64, [_c_i, _c_i]),
    "trex_plan_build": (_c_i, [_p, _c_i, _c_i, _p, _p]),
    "trex_workspace_bytes": (_c_i64, [_c_i, _c_i, _c_i, _c_i]),
    "trex_sankoff_fwd": (_c_i, [_p, _c_i, _p, _p, _c_i, _c_i, _c_i, _c_i, _c_f, _c_u,
                                _p, _p, _p, _p, _c_i64, _p]),
    "trex_sankoff_bwd": (_c_i, [_p, _c_i, _p, _p, _c_i, _c_i, _c_i, _c_i, _c_f, _c_u,
                                _p, _p, _p, _p, _p, _p, _c_i64, _p]),
    "trex_workspace_init": (_c_i, [_p, _c_i64, _p]),
    "trex_sankoff_fwd_bwd": (_c_i, [_p, _c_i, _p, _p, _c_i, _c_i, _c_i, _c_i, _c_f, _c_u,
                                    _p, _p, _p, _p, _p, _p, _p, _p, _c_i64, _p]),
    "trex_sankoff_backtrack": (_c_i, [_p, _c_i, _p, _p, _c_i, _c_i, _c_i, _c_i, _p, _p]),
    "trex_dp_to_trex_layout": (_c_i, [_p, _p, _c_i, _c_i, _c_i, _c_i, _p, _p]),
    "trex_dp_site_major": (_c_i, [_c_i]),
    # multi-GPU exchange (RCCL, dlopen'ed on first use)
    "trex_comm_unique_id_bytes": (_c_i, []),
    "trex_comm_get_unique_id": (_c_i, [_p]),
    "trex_comm_init": (_c_i, [ctypes.POINTER(_p), _c_i, _p, _c_i, _c_i]),
    "trex_comm_destroy": (_c_i, [_p]),
    "trex_allreduce_sum": (_c_i, [_p, _c_i, _c_i, _p, _p]),
    # raw-table run_dp / backtrack_sankoff_jit
    "trex_run_dp": (_c_i, [_p, _c_i, _c_i, _c_i, _p, _c_i, _p, _p, _p, _p]),
    "trex_backtrack_workspace_bytes": (_c_i64, [_c_i, _c_i]),
    "trex_backtrack_generic": (_c_i, [_c_i, _p, _p, _p, _c_i, _c_i, _c_i, _c_i, _p, _p, _c_i64,
                                      _c_i64, _p, _p]),
    "trex_dp_root_total": (_c_i, [_p, _c_i, _c_i, _c_i, _p, _p, _p]),
    # tree-cost path
    "trex_tree_discretize": (_c_i, [_p, _c_i, _c_i, _c_i, _p, _p]),
    "trex_tree_update_seq": (_c_i, [_p, _c_i, _c_i, _c_i, _c_f, _p, _p]),
    "trex_tree_update_seq_bwd": (_c_i, [_p, _p, _c_i, _c_i, _c_i, _c_f, _p, _p]),
    "trex_tree_update_tree": (_c_i, [_p, _p, _p, _c_i, _c_i, _c_f, _p, _p]),
    "trex_tree_update_tree_bwd": (_c_i, [_p, _p, _p, _c_i, _c_i, _c_f, _p, _p]),
    "trex_tree_workspace_bytes": (_c_i64, [_c_i, _c_i64]),
    "trex_tree_surrogate": (_c_i, [_p, _p, _c_i, _c_i64, _p, _p, _p, _p, _p, _c_i64, _p]),
    "trex_tree_gram": (_c_i, [_p, _c_i, _c_i64, _p, _p, _c_i64, _p]),
    "trex_tree_gram_skip": (_c_i, [_p, _c_i, _c_i64, _c_i, _p, _p, _c_i64, _p]),
    "trex_tree_surrogate_combine": (_c_i, [_p, _p, _c_i, _p, _p, _p, _p, _p]),
    "trex_tree_mf": (_c_i, [_p, _p, _c_i, _c_i64, _p, _p]),
    # ragged batches
    "trex_ragged_plan_ints": (_c_i64, [_c_i, _p, _p]),
    "trex_ragged_plan_build": (_c_i, [_p, _p, _p, _c_i, _p, _p]),
    "trex_ragged_workspace_bytes": (_c_i64, [_c_i64, _c_i]),
    "trex_sankoff_ragged": (_c_i, [_c_i, _p, _c_i, _c_i, _c_i, _c_i64, _p, _p, _c_i, _c_f, _c_u,
                                   _p, _p, _p, _p, _p, _p, _p, _p, _c_i64, _p]),
    "trex_sankoff_ragged_backtrack": (_c_i, [_p, _c_i, _c_i64, _c_i64, _c_i, _p, _p, _c_i, _p,
                                             _p]),
    # NK landscape-aware loss
    "trex_nk_parental_logits": (_c_i, [_p, _p, _c_i, _c_i, _c_i, _p, _c_i, _p, _p, _p]),
    "trex_nk_plan_ints": (_c_i64, [_c_i, _c_i, _c_i]),
    "trex_nk_plan_build": (_c_i, [_p, _c_i, _p, _c_i, _c_i, _p, _p]),
    "trex_nk_workspace_bytes": (_c_i64, [_c_i, _c_i, _c_i, _c_i, _c_i]),
    "trex_nk_landscape_loss": (_c_i, [_p, _c_i, _p, _c_i, _c_i, _c_i, _p, _c_i, _p, _p, _c_f,
                                      _c_f, _c_i, _p, _p, _p, _p, _p, _c_i64, _p]),
    "trex_tree_mf_rows": (_c_i, [_p, _p, _c_i, _c_i64, _c_i, _c_i, _p, _p]),
    "trex_tree_gram_skip_x3": (_c_i, [_p, _c_i, _c_i64, _c_i, _c_f, _p, _p, _c_i64, _p]),
    "trex_tree_gram_mirror": (_c_i, [_p, _c_i, _c_i, _p]),
    "trex_tree_mf_rows_x3": (_c_i, [_p, _p, _c_i, _c_i64, _c_i, _c_i, _c_f, _c_f, _p, _p]),
    # leaf-code MF operand (exact one-hot leaf rows, Q = 4)
    "trex_tree_leaf_code_rows": (_c_i, [_c_i]),
    "trex_tree_leaf_codes_bytes": (_c_i64, [_c_i, _c_i]),
    "trex_tree_leaf_codes": (_c_i, [_p, _c_i, _c_i, _c_i, _p, _c_i64, _p, _p]),
    "trex_tree_mf_rows_x3_codes": (_c_i, [_p, _p, _c_i, _c_i64, _c_i, _c_i, _c_f, _c_f, _p,
                                          _c_i64, _c_i, _c_i, _p, _p]),
    "trex_tree_surrogate_constraint": (_c_i, [_p, _p, _c_i, _c_f, _c_f, _p, _p, _p, _p, _c_f, _p,
                                              _c_i, _p, _p]),
    "trex_tree_split_x3": (_c_i, [_p, _c_i, _c_i, _c_i, _c_f, _p, _c_i, _p]),
    "trex_tree_gram_skip_x3p": (_c_i, [_p, _c_i, _c_i64, _c_i, _c_f, _p, _p, _c_i64, _p]),
    "trex_tree_gram_skip_x3p_codes": (_c_i, [_p, _c_i, _c_i64, _c_i, _c_f, _p, _c_i64, _c_i,
                                             _c_i, _p, _p, _c_i64, _p]),
    "trex_tree_mf_rows_x3p": (_c_i, [_p, _c_i, _p, _c_i, _c_i64, _c_i, _c_i, _c_f, _c_f, _p,
                                     _c_i64, _c_i, _c_i, _p, _p]),
    "trex_adam_seq_update_step_x3p": (_c_i, [_p, _c_i, _c_i, _c_i, _c_f, _c_f, _p, _p, _p, _c_i,
                                             _c_f, _c_f, _c_f, _c_f, _p, _c_f, _p, _p]),
    "trex_tree_update_tree_bwd_adam": (_c_i, [_p, _p, _p, _c_i, _c_i, _c_f, _p, _p, _p, _p, _c_i,
                                              _p, _c_f, _c_f, _c_f, _c_f, _p]),
    "trex_tree_soft_cost": (_c_i, [_p, _p, _p, _c_i, _c_i, _c_i, _c_i, _p, _p, _p, _c_i64, _p]),
    "trex_tree_constraint": (_c_i, [_p, _c_i, _c_f, _c_f, _p, _c_i, _p, _p, _p]),
    "trex_tree_compute_cost": (_c_i, [_p, _p, _p, _c_i, _c_i, _c_i, _p, _p, _p]),
    "trex_adam_step": (_c_i, [_p, _p, _p, _p, _c_i64, _c_i, _c_f, _c_f, _c_f, _c_f, _p, _c_i,
                              _c_f, _p]),
    "trex_sq_norm_parts": (_c_i, [_p, _c_i64, _p, _c_i, _p]),
    "trex_optax_step": (_c_i, [_c_i, _p, _p, _p, _p, _c_i64, _c_i, _c_f, _c_f, _c_f, _c_f, _c_f,
                               _p, _c_i, _c_f, _p]),
    "trex_adam_seq_update_step": (_c_i, [_p, _c_i, _c_i, _c_i, _c_f, _c_f, _p, _p, _p, _c_i, _c_f,
                                         _c_f, _c_f, _c_f, _p, _p]),
    "trex_adam_seq_step": (_c_i, [_p, _p, _c_i, _c_i, _c_i, _c_f, _p, _p, _p, _c_i, _c_f, _c_f,
                                  _c_f, _c_f, _p, _p]),
    # device step state: graph-capturable optimisation loops (ABI v7)
    "trex_step_state_bytes": (_c_i, []),
    "trex_step_advance": (_c_i, [_p, _c_f, _c_f, _p, _c_i64, _p]),
    "trex_adam_step_dev": (_c_i, [_p, _p, _p, _p, _c_i64, _p, _c_f, _c_f, _c_f, _c_f, _p, _c_i,
                                  _c_f, _p]),
    "trex_optax_step_dev": (_c_i, [_c_i, _p, _p, _p, _p, _c_i64, _p, _c_f, _c_f, _c_f, _c_f,
                                   _c_f, _p, _c_i, _c_f, _p]),
    "trex_adam_seq_update_step_dev": (_c_i, [_p, _c_i, _c_i, _c_i, _p, _p, _p, _p, _c_f, _c_f,
                                             _c_f, _c_f, _p, _p]),
    "trex_tree_constraint_dev": (_c_i, [_p, _c_i, _c_f, _p, _p, _c_i, _p, _p, _p]),
    "trex_gumbel_noise": (_c_i, [ctypes.c_uint64, _p, _c_i64, _p, _p]),
    # synthetic data on the device
    "trex_datagen_workspace_bytes": (_c_i64, [_c_i, _c_i]),
    "trex_datagen_groundtruth": (_c_i, [ctypes.c_uint64, _c_i, _c_i, _c_i, _c_i, _p, _p, _c_i64,
                                        _p]),
    "trex_datagen_uniform_states": (_c_i, [ctypes.c_uint64, _c_i64, _c_i, _p, _p]),
    "trex_datagen_nk_tree": (_c_i, [ctypes.c_uint64, _c_i, _c_i, _c_i, _c_i, _p, _p, _p, _p, _p, _c_i,
                                    _c_f, _c_f, _c_f, _c_i, _p, _p]),
}


class TrexError(RuntimeError):
    """A libtrexhip.so call returned a negative TREX_E_* code."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


_LIB = None


def lib() -> ctypes.CDLL:
    """Load libtrexhip.so once; raise loudly when it is absent."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"libtrexhip.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` -- there is no CPU fallback")
        handle = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = handle
    return _LIB


def check(rc: int) -> None:
    if rc != TREX_OK:
        raise TrexError(rc, lib().trex_last_error().decode(errors="replace"))


def ptr(t) -> int | None:
    """Device/host pointer of a torch tensor or numpy array (None passes NULL)."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    return t.ctypes.data


def stream_handle(device=None) -> int | None:
    import torch

    return torch.cuda.current_stream(device).cuda_stream
