"""Data parallelism for the two sharded paths (one process per GPU).

C4 (Sankoff): tree-batch sharding, one all-reduce of [dC, loss].
C5 (tree cost): site sharding, one all-reduce of the N x N Gram matrix.


Trees (and sites) are independent in Sankoff (src/trex/sankoff.py:97 vmaps
sites; trex has no batch-of-trees axis or collectives).  The build shards
the tree batch in contiguous blocks across ranks; the ONLY exchange is the sum
of the cost-matrix gradient and the loss, packed into one Q*Q+1 fp32 buffer
and all-reduced once per step (RCCL over xGMI with backend "nccl"; gloo on
CPU in tests).  68 bytes at Q=4: latency-bound, so it is one call, fused.
"""

from __future__ import annotations


def shard_bounds(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced block [lo, hi) of n_items for this rank."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(n_items, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class GradReducer:
    """Packs (d_cost, sum of tree scores) and all-reduces them in one call."""

    def __init__(self, n_states: int, device, group=None):
        import torch

        self.Q = n_states
        self.group = group
        self.buf = torch.zeros(n_states * n_states + 1, dtype=torch.float32, device=device)

    def __call__(self, d_cost, tree_score):
        import torch.distributed as dist

        q2 = self.Q * self.Q
        self.buf[:q2].copy_(d_cost.reshape(-1))
        self.buf[q2:].copy_(tree_score.sum().reshape(1))
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(self.buf, group=self.group)
        return self.buf[:q2].view(self.Q, self.Q), self.buf[q2]


class GramReducer:
    """C5 site sharding: the surrogate's only cross-site term.

    compute_surrogate_cost (src/trex/tree.py:199-209) depends on the sites only
    through G = S S^T (with E = diag G), a sum over sites; each rank computes
    G over its block of sites and one all-reduce makes every rank's G the
    full one: the whole N x N matrix once (1.04 MB at N = 511), then per step
    only the rows the step recomputes (``G[row0:]``, the ancestor rows x all
    columns: 0.52 MB; TreeOptimizer mirrors them into the leaf rows).  The combine (value, dA,
    M = diag(r+c) - (A+A^T)), the tree_params gradient and their Adam update
    are then identical on all ranks; dS = M S_local stays local.
    """

    def __init__(self, group=None):
        self.group = group
        self.calls = 0  # all-reduces issued and their payload (bench.py reports
        self.bytes = 0  # the per-step Gram exchange from these)

    def __call__(self, G):
        import torch.distributed as dist

        if not G.is_contiguous():
            raise ValueError("GramReducer: G (or its row block) must be contiguous")
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(G, group=self.group)
            self.calls += 1
            self.bytes += G.numel() * G.element_size()
        return G


class NativeComm:
    """The C ABI's RCCL exchange (trex_comm_* / trex_allreduce_sum in
    include/trex_hip.h): what a binding without torch.distributed uses for
    the sharded paths' one all-reduce.  ``unique_id`` comes from rank 0's
    ``NativeComm.new_unique_id()`` and is shared out of band."""

    def __init__(self, nranks: int, rank: int, unique_id: bytes, device_index: int):
        import ctypes

        from ._lib import check, lib

        self.dev = int(device_index)
        self.comm = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(unique_id), lib().trex_comm_unique_id_bytes())
        check(lib().trex_comm_init(ctypes.byref(self.comm), int(nranks), buf, int(rank), self.dev))

    @staticmethod
    def new_unique_id() -> bytes:
        import ctypes

        from ._lib import check, lib

        n = lib().trex_comm_unique_id_bytes()
        buf = ctypes.create_string_buffer(n)
        check(lib().trex_comm_get_unique_id(buf))
        return buf.raw

    def all_reduce_sum(self, t):
        """In-place sum over ranks of a contiguous fp32 device tensor, on
        torch's current stream."""
        import torch

        from ._lib import check, lib, stream_handle

        if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
            raise ValueError("all_reduce_sum takes a contiguous fp32 device tensor")
        check(lib().trex_allreduce_sum(t.data_ptr(), t.numel(), self.dev, self.comm,
                                       stream_handle(t.device)))
        return t

    def close(self):
        from ._lib import check, lib

        if self.comm:
            check(lib().trex_comm_destroy(self.comm))
            self.comm = None
