"""trex_amd -- MI355X-native engine for trex's batched Sankoff / tree-cost path.

Mirrors the public functions of maraxen/trex ``trex.sankoff`` (and, as they
land, ``trex.tree``) on top of hand-written HIP kernels for gfx950 in
``libtrexhip.so`` (C ABI: include/trex_hip.h).  See DESIGN.md.
"""

from ._lib import LIB_PATH, TrexError, lib  # noqa: F401
from .sankoff import (  # noqa: F401
    SankoffEngine,
    backtrack_sankoff_jit,
    leaf_codes,
    run_dp,
    run_sankoff,
    sankoff_value_and_grad,
    vectorized_dp,
    vmapped_backtrack,
)
from .topology import (  # noqa: F401
    TreePlan,
    children_from_adjacency,
    create_balanced_binary_tree,
    random_topologies,
)

__all__ = [
    "LIB_PATH", "TrexError", "lib", "SankoffEngine", "leaf_codes", "run_sankoff", "run_dp",
    "vectorized_dp", "backtrack_sankoff_jit", "vmapped_backtrack",
    "sankoff_value_and_grad", "TreePlan", "children_from_adjacency",
    "create_balanced_binary_tree", "random_topologies",
]
