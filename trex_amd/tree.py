"""trex's ``tree`` module on MI355X.

Mirrors maraxen/trex ``src/trex/tree.py``:
* ``discretize_tree_topology`` (:31-47), ``update_tree`` (:50-107),
  ``update_seq`` (:110-130);
* ``enforce_graph_constraints`` (:133-160), ``compute_surrogate_cost``
  (:163-209), ``compute_soft_cost`` (:212-266), ``compute_cost`` (:269-296);
* ``compute_loss`` (:299-361).

It adds what the reference gets from jax.grad and optax: ``loss_and_grad``
(analytic reverse mode on the same kernels) and ``Adam`` (optax.adam /
clip_by_global_norm semantics, src/trex/evals/benchmark.py:41-72).

One interface change: ``update_tree`` takes its Gumbel noise explicitly
(``noise`` instead of a JAX PRNG key), since trex's threefry stream
(tree.py:71) is JAX-specific.  ``gumbel_noise`` draws one with torch.
All arithmetic runs in libtrexhip.so.
"""

from __future__ import annotations

import os

import numpy as np

from ._lib import check, lib, ptr, stream_handle


def _torch():
    import torch

    return torch


def _dev(x, device=None):
    torch = _torch()
    t = torch.as_tensor(x)
    if device is None:
        device = t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())
    return t.to(device=device, dtype=torch.float32).contiguous()


_WS: dict = {}


def _workspace(N, K, device):
    torch = _torch()
    nbytes = int(lib().trex_tree_workspace_bytes(N, K))
    key = str(device)
    ws = _WS.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _WS[key] = ws
    return ws


def gumbel_noise(shape, generator=None, device=None):
    """Standard Gumbel noise (what jax.random.gumbel draws at tree.py:71)."""
    torch = _torch()
    device = device or torch.device("cuda", torch.cuda.current_device())
    u = torch.rand(shape, generator=generator, device=device, dtype=torch.float32)
    return -torch.log(-torch.log(u.clamp_min(1e-20)))


def step_state(device, count: int = 0):
    """A device step state (trex_step_advance, include/trex_hip.h) holding
    `count` steps already taken."""
    torch = _torch()
    nwords = int(lib().trex_step_state_bytes()) // 4
    st = torch.zeros(nwords, dtype=torch.int32, device=device)
    if count:
        st[0] = int(count)
    return st


def gumbel_noise_step(seed: int, step: int, shape, device=None, out=None):
    """The Gumbel noise a device loop draws at (1-based) step `step`
    (trex_gumbel_noise: a pure function of seed, step and index)."""
    torch = _torch()
    device = device or torch.device("cuda", torch.cuda.current_device())
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=device)
    st = step_state(device, step)
    check(lib().trex_gumbel_noise(int(seed) & (2**64 - 1), ptr(st), out.numel(), ptr(out),
                                  stream_handle(device)))
    return out


# ---------------------------------------------------------------------------
# PRNG keys (the reference's `key` arguments)
# ---------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


class PRNGKey:
    """Stand-in for a ``jax.random.PRNGKey`` where the reference takes a key
    (update_tree tree.py:71, compute_loss tree.py:337): a 64-bit seed whose
    Gumbel draw is ``trex_gumbel_noise`` (a pure function of seed, step and
    index), and ``split`` derives children by splitmix64.  JAX's threefry
    stream itself cannot be reproduced without JAX, so draws differ from
    trex's for the same integer seed; the call shapes and the determinism
    (same key -> same noise, split keys independent) are the reference's."""

    __slots__ = ("seed",)

    def __init__(self, seed: int):
        self.seed = int(seed) & _M64

    def __repr__(self):
        return f"PRNGKey({self.seed:#x})"

    def __eq__(self, other):
        return isinstance(other, PRNGKey) and other.seed == self.seed

    def __hash__(self):
        return hash(("trex_amd.PRNGKey", self.seed))


def split(key: PRNGKey, num: int = 2):
    """``jax.random.split(key, num)``'s role: ``num`` child keys."""
    return tuple(PRNGKey(_splitmix64(key.seed ^ _splitmix64(i + 1))) for i in range(int(num)))


def gumbel(key: PRNGKey, shape, device=None):
    """Standard Gumbel noise of ``shape`` drawn from ``key`` on the device."""
    return gumbel_noise_step(key.seed, 1, shape, device)


def _tree_noise(noise, shape, device):
    """update_tree's noise argument: a PRNGKey draws, a tensor is the noise."""
    if isinstance(noise, PRNGKey):
        return gumbel(noise, shape, device)
    return _dev(noise, device) if noise is not None else None


# ---------------------------------------------------------------------------
# topology / sequences
# ---------------------------------------------------------------------------
def discretize_tree_topology(adjacency, n_nodes: int):
    """one_hot(argmax(adjacency, 1)) (tree.py:46-47), first index on ties."""
    torch = _torch()
    A = _dev(adjacency)
    out = torch.empty((A.shape[0], n_nodes), dtype=torch.float32, device=A.device)
    check(lib().trex_tree_discretize(ptr(A), A.shape[0], A.shape[1], n_nodes, ptr(out),
                                     stream_handle(A.device)))
    return out


def update_tree(noise, params, temperature: float = 1.0, gates=None):
    """Relaxed topology: row softmax of the masked logits (tree.py:50-107).
    ``noise``: the Gumbel noise (n_nodes - 1, n_anc), or a PRNGKey to draw it
    from (the reference's ``key``), or None (no noise)."""
    torch = _torch()
    theta = _dev(params["tree_params"])
    n_m1, n_anc = theta.shape
    N = n_m1 + 1
    dev = theta.device
    nz = _tree_noise(noise, (n_m1, n_anc), dev)
    gt = _dev(gates, dev) if gates is not None else None
    A = torch.empty((N, N), dtype=torch.float32, device=dev)
    check(lib().trex_tree_update_tree(ptr(theta), ptr(nz), ptr(gt), N, n_anc, float(temperature),
                                      ptr(A), stream_handle(dev)))
    return A


def _ancestors(params):
    torch = _torch()
    anc = params["ancestors"]
    if isinstance(anc, (list, tuple)):
        anc = torch.stack([torch.as_tensor(a) for a in anc])
    return _dev(anc)


def update_seq(params, sequences, temperature: float = 1.0):
    """S[n_leaf:] = softmax(ancestors * T) (tree.py:127-130)."""
    anc = _ancestors(params)
    S = _dev(sequences, anc.device).clone()
    n_leaf = (S.shape[0] + 1) // 2
    n_anc, L, Q = anc.shape
    if S.shape[0] - n_leaf != n_anc or tuple(S.shape[1:]) != (L, Q):
        raise ValueError("ancestors must be (n_nodes - (n_nodes+1)//2, L, Q)")
    check(lib().trex_tree_update_seq(ptr(anc), n_anc, L, Q, float(temperature), ptr(S[n_leaf:]),
                                     stream_handle(S.device)))
    return S


def enforce_graph_constraints(adjacency, scaling_factor: float):
    """scale * sum_cols (sum_rows A[:-1, -n_anc:] - 2)^2 (tree.py:156-160)."""
    torch = _torch()
    A = _dev(adjacency)
    out = torch.empty((1,), dtype=torch.float32, device=A.device)
    ws = _workspace(A.shape[0], 1, A.device)
    check(lib().trex_tree_constraint(ptr(A), A.shape[0], float(scaling_factor), 1.0, ptr(out), 0,
                                     None, ptr(ws), stream_handle(A.device)))
    return out[0]


# ---------------------------------------------------------------------------
# tree costs
# ---------------------------------------------------------------------------
def compute_surrogate_cost(sequences, adjacency):
    """0.5 * sum_ij A_ij ||S_i - S_j||^2 (tree.py:163-209)."""
    torch = _torch()
    S = _dev(sequences)
    A = _dev(adjacency, S.device)
    N = S.shape[0]
    K = S[0].numel()
    out = torch.empty((1,), dtype=torch.float32, device=S.device)
    ws = _workspace(N, K, S.device)
    check(lib().trex_tree_surrogate(ptr(S), ptr(A), N, K, ptr(out), None, None, None, ptr(ws),
                                    ws.numel(), stream_handle(S.device)))
    return out[0]


def surrogate_cost_and_grads(sequences, adjacency):
    """(cost, dS, dA) of compute_surrogate_cost: dS = (diag(r+c) - (A+A^T)) S,
    dA = (E_i + E_j)/2 - G_ij."""
    torch = _torch()
    S = _dev(sequences)
    A = _dev(adjacency, S.device)
    N = S.shape[0]
    K = S[0].numel()
    out = torch.empty((1,), dtype=torch.float32, device=S.device)
    dS = torch.empty_like(S)
    dA = torch.empty_like(A)
    ws = _workspace(N, K, S.device)
    check(lib().trex_tree_surrogate(ptr(S), ptr(A), N, K, ptr(out), ptr(dS), ptr(dA), None,
                                    ptr(ws), ws.numel(), stream_handle(S.device)))
    return out[0], dS, dA


def compute_soft_cost(sequences, adjacency, cost_matrix=None):
    """Weighted variant (tree.py:212-266): C None, (Q,) diagonal or (Q, Q)."""
    torch = _torch()
    S = _dev(sequences)
    A = _dev(adjacency, S.device)
    N, L, Q = S.shape
    ckind = 0
    C = None
    W = None
    if cost_matrix is not None:
        C = _dev(cost_matrix, S.device)
        ckind = 1 if C.ndim == 1 else 2
        W = torch.empty_like(S)
    out = torch.empty((1,), dtype=torch.float32, device=S.device)
    ws = _workspace(N, L * Q, S.device)
    check(lib().trex_tree_soft_cost(ptr(S), ptr(A), ptr(C), ckind, N, L, Q, ptr(out), ptr(W),
                                    ptr(ws), ws.numel(), stream_handle(S.device)))
    return out[0]


def compute_cost(sequences, adjacency, substitution_matrix):
    """Exact cost of a labelled tree (tree.py:286-296)."""
    torch = _torch()
    S = _dev(sequences)
    A = _dev(adjacency, S.device)
    C = _dev(substitution_matrix, S.device)
    N, L, Q = S.shape
    out = torch.empty((1,), dtype=torch.float32, device=S.device)
    ws = _workspace(N, 1, S.device)
    check(lib().trex_tree_compute_cost(ptr(S), ptr(A), ptr(C), N, L, Q, ptr(out), ptr(ws),
                                       stream_handle(S.device)))
    return out[0]


# ---------------------------------------------------------------------------
# loss and its gradient
# ---------------------------------------------------------------------------
def loss_and_grad(noise, params, sequences, temperature: float, adjacency=None, *,
                  graph_constraint_scale: float = 10.0, fix_seqs: bool = False,
                  fix_tree: bool = False):
    """compute_loss (tree.py:336-342) and d loss / d params.

    update_tree runs at temperature 1.0: compute_loss does not pass T to it
    (tree.py:338).  ``noise``: update_tree's Gumbel noise, or a PRNGKey,
    split as the reference splits its key (tree.py:337: the second half
    draws the noise).  Returns (loss, {"tree_params", "ancestors"}).
    """
    if isinstance(noise, PRNGKey):
        noise = split(noise)[1]
    torch = _torch()
    theta = _dev(params["tree_params"])
    anc = _ancestors(params)
    dev = theta.device
    st = stream_handle(dev)
    S = _dev(sequences, dev) if fix_seqs else update_seq({"ancestors": anc}, sequences,
                                                         temperature)
    A = _dev(adjacency, dev) if fix_tree else update_tree(noise, {"tree_params": theta}, 1.0)
    N = S.shape[0]
    K = S[0].numel()
    loss = torch.empty((1,), dtype=torch.float32, device=dev)
    dS = torch.empty_like(S)
    dA = torch.empty_like(A)
    ws = _workspace(N, K, dev)
    check(lib().trex_tree_surrogate(ptr(S), ptr(A), N, K, ptr(loss), ptr(dS), ptr(dA), None,
                                    ptr(ws), ws.numel(), st))
    # + T * constraint (value and gradient accumulated into dA)
    check(lib().trex_tree_constraint(ptr(A), N, float(graph_constraint_scale),
                                     float(temperature), ptr(loss), 1, ptr(dA), ptr(ws), st))
    grads = {"tree_params": torch.zeros_like(theta), "ancestors": torch.zeros_like(anc)}
    if not fix_tree and theta.shape[1] > 0:
        check(lib().trex_tree_update_tree_bwd(ptr(A), ptr(dA), None, N, theta.shape[1], 1.0,
                                              ptr(grads["tree_params"]), st))
    if not fix_seqs:
        n_leaf = (N + 1) // 2
        n_anc, L, Q = anc.shape
        check(lib().trex_tree_update_seq_bwd(ptr(S[n_leaf:]), ptr(dS[n_leaf:]), n_anc, L, Q,
                                             float(temperature), ptr(grads["ancestors"]), st))
    return loss[0], grads


def compute_loss(noise, params, sequences, _metadata, temperature: float, adjacency, *,
                 graph_constraint_scale: float = 10.0, verbose: bool = False,
                 fix_seqs: bool = False, fix_tree: bool = False):
    """Total loss (tree.py:299-361); ``noise`` is a PRNGKey (split as the
    reference splits its key) or update_tree's noise itself."""
    loss, _ = loss_and_grad(noise, params, sequences, temperature, adjacency,
                            graph_constraint_scale=graph_constraint_scale, fix_seqs=fix_seqs,
                            fix_tree=fix_tree)
    return loss


# ---------------------------------------------------------------------------
# optimiser (optax semantics)
# ---------------------------------------------------------------------------
class Adam:
    """optax.adam(lr, b1, b2, eps) [chained after clip_by_global_norm(clip)].

    Updates the parameter tensors in place with one fused kernel per tensor.

    ``sharded``: names of tensors whose gradient is split over the ranks of
    ``group`` (site sharding: each rank holds a block of the tensor).  The
    global norm of clip_by_global_norm then sums their squared-norm partials
    over the ranks (one all-reduce of 512 fp64 partials per sharded tensor);
    the other tensors are replicated and counted once.
    """

    def __init__(self, params: dict, lr: float, b1=0.9, b2=0.999, eps=1e-8, clip_norm=None, *,
                 sharded=(), group=None):
        torch = _torch()
        self.lr, self.b1, self.b2, self.eps, self.clip = lr, b1, b2, eps, clip_norm
        self.sharded = frozenset(sharded)
        self.group = group
        self.mu = {k: torch.zeros_like(v) for k, v in params.items()}
        self.nu = {k: torch.zeros_like(v) for k, v in params.items()}
        self.count = 0
        dev = next(iter(params.values())).device
        self.parts = torch.zeros(512 * max(1, len(params)), dtype=torch.float64, device=dev)
        # the step count and bias corrections live on the device (advanced by
        # a kernel each step), so a step captured in a hipGraph replays with
        # the right count (trex_step_advance; bitwise the host-count update)
        self.state = step_state(dev)
        # TreeOptimizer's eager step counts on the host only (no launch);
        # sync_state() brings the device record up to date before any
        # device-side use
        self._state_stale = False

    def sync_state(self):
        """Reset the device step record to the host count, in place (a
        captured graph keeps its pointer), when eager steps left it behind."""
        if self._state_stale:
            self.state.zero_()
            self.state[0] = int(self.count)
            self._state_stale = False

    def state_dict(self) -> dict:
        """Host copies of the optimiser state: step count, first / second
        moments (optax's ScaleByAdamState)."""
        return {"count": int(self.count),
                "mu": {k: v.detach().cpu().clone() for k, v in self.mu.items()},
                "nu": {k: v.detach().cpu().clone() for k, v in self.nu.items()}}

    def load_state_dict(self, sd: dict):
        """Restore a ``state_dict``; the device step record restarts at its
        count (the next step recomputes the bias corrections from it)."""
        for name in ("mu", "nu"):
            mine = getattr(self, name)
            for k, v in sd[name].items():
                if k not in mine or tuple(mine[k].shape) != tuple(v.shape):
                    raise ValueError(f"Adam.load_state_dict: {name}[{k!r}] does not match")
                mine[k].copy_(v.to(mine[k].device, dtype=mine[k].dtype))
        self.count = int(sd["count"])
        self._state_stale = True
        self.sync_state()

    def step(self, params: dict, grads: dict):
        """One update; launches only kernels (graph-capturable unless the
        clip norm is all-reduced over a process group)."""
        self.sync_state()
        self.count += 1
        st = stream_handle(next(iter(params.values())).device)
        check(lib().trex_step_advance(ptr(self.state), float(self.b1), float(self.b2), None, 0,
                                      st))
        keys = sorted(params)
        nparts = 0
        if self.clip is not None:
            for i, k in enumerate(keys):
                check(lib().trex_sq_norm_parts(ptr(grads[k]), grads[k].numel(),
                                               ptr(self.parts[512 * i:]), 512, st))
                if k in self.sharded:
                    import torch.distributed as dist

                    if dist.is_available() and dist.is_initialized():
                        dist.all_reduce(self.parts[512 * i:512 * (i + 1)], group=self.group)
            nparts = 512 * len(keys)
        for k in keys:
            p, g = params[k], grads[k]
            if not (p.is_contiguous() and g.is_contiguous()):
                raise ValueError("params and grads must be contiguous")
            check(lib().trex_adam_step_dev(ptr(p), ptr(g), ptr(self.mu[k]), ptr(self.nu[k]),
                                           p.numel(), ptr(self.state), float(self.lr),
                                           float(self.b1), float(self.b2), float(self.eps),
                                           ptr(self.parts) if nparts else None, nparts,
                                           float(self.clip or 0.0), st))


class TreeOptimizer:
    """Device-resident compute_loss + optax-Adam step: the C5 loop.

    Joint optimisation of tree_params and ancestor logits as in
    tests/test_convergence.py:208-261 (loss = surrogate(update_seq(params, T),
    update_tree(params, 1.0)) + T * constraint, Adam(lr)).  Buffers are
    allocated once; ``step`` launches only HIP kernels (graph-capturable).

    Site sharding (``group``): each rank holds a contiguous block of sites
    (its leaf one-hot rows and ancestor logits for those sites).  The only
    exchange is an all-reduce of the Gram rows that change (the ancestor
    rows x all columns; the leaf x leaf block is reduced once at
    construction and cached); every rank then
    computes the same loss, dA and tree_params update, and updates its own
    ancestor logits.  With ``clip_norm`` (the evals path's
    clip_by_global_norm(1.0), src/trex/evals/benchmark.py:70-71) one more
    all-reduce sums the ancestors' squared-norm partials over the ranks.

    ``gemm``: "x3" (default) runs the two N x N x L*Q GEMMs as f16x3 split
    products on f16 MFMA (``trex_tree_gram_skip_x3`` / ``trex_tree_mf_rows_x3``;
    S is a softmax / one-hot, |S| <= 1, and M = diag(r+c) - (A+A^T) with
    softmax rows, |M| <= N+1, inside their contract), "f32" on f32 MFMA.
    Both meet the same rtol 1e-5 bar against the fp64 oracle.
    """

    def __init__(self, sequences, params: dict, lr: float = 0.01, *,
                 graph_constraint_scale: float = 10.0, clip_norm=None, group=None,
                 gemm: str = "x3"):
        torch = _torch()
        # (N, L, Q): leaf rows fixed, ancestor rows rewritten by each step --
        # except in pre-split mode (x3, Q = 4, no clipping), where the steps
        # keep only S16's ancestor rows current and S's go stale after the
        # first step: read sequences() for the current softmaxes
        self.S = _dev(sequences).clone()
        dev = self.S.device
        self.params = {"tree_params": _dev(params["tree_params"], dev).clone(),
                       "ancestors": _ancestors(params).to(dev).clone()}
        self.N, self.L, self.Q = self.S.shape
        self.K = self.L * self.Q
        self.n_leaf = (self.N + 1) // 2
        self.n_anc = self.N - self.n_leaf
        self.scale = float(graph_constraint_scale)
        self.group = group
        self.reducer = None
        if group is not None:
            from .distributed import GramReducer

            self.reducer = GramReducer(group)
        f32 = dict(dtype=torch.float32, device=dev)
        self.A = torch.empty((self.N, self.N), **f32)
        self.G = torch.empty((self.N, self.N), **f32)
        self.M = torch.empty((self.N, self.N), **f32)
        self.dA = torch.empty((self.N, self.N), **f32)
        self.dS = torch.empty_like(self.S)
        self.loss = torch.zeros((1,), **f32)
        self.grads = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.ws = torch.empty(int(lib().trex_tree_workspace_bytes(self.N, self.K)),
                              dtype=torch.uint8, device=dev)
        # with site sharding the ancestor logits are this rank's block of
        # sites: clip_by_global_norm sums their squared norm over the ranks
        self.opt = Adam(self.params, lr, clip_norm=clip_norm,
                        sharded=("ancestors",) if group is not None else (), group=group)
        self._s_temperature = None  # temperature the S ancestor rows were computed with
        if gemm not in ("x3", "f32"):
            raise ValueError("gemm must be 'x3' or 'f32'")
        # the split-product GEMMs load 16-B row pieces: K = L*Q % 4 == 0 (a
        # ragged last K chunk is masked in the kernels, so a site shard of
        # any length works when Q % 4 == 0)
        self.gemm = gemm
        if gemm == "x3" and self.K % 4 != 0:
            import warnings

            warnings.warn(f"TreeOptimizer: K = L*Q = {self.K} is not a multiple of 4; the f16x3 "
                          "GEMMs need 16-B aligned rows, running the f32 MFMA GEMMs instead",
                          RuntimeWarning, stacklevel=2)
            self.gemm = "f32"
        # the leaf x leaf block of G = S S^T is constant (leaf rows are data):
        # computed once here (all-reduced once under site sharding), skipped
        # by every step's Gram.  Rows [g_row0, N) are recomputed each step;
        # under sharding only they are all-reduced, then mirrored into the
        # leaf rows' ancestor columns (trex_tree_gram_mirror).
        check(lib().trex_tree_gram(ptr(self.S), self.N, self.K, ptr(self.G), ptr(self.ws),
                                   self.ws.numel(), stream_handle(dev)))
        if self.reducer is not None:
            self.reducer(self.G)
        self.skip_rows = self.n_leaf
        self.g_row0 = (self.skip_rows // 64) * 64
        # exact one-hot leaf rows (Q = 4): the x3 MF reads their codes
        # instead of the f32 rows (bitwise the same dS, trex_tree_leaf_codes);
        # TREX_LEAF_CODES=0 keeps the f32 rows
        self.codes = None
        if (self.gemm == "x3" and self.Q == 4 and lib().trex_tree_leaf_code_rows(self.n_leaf) > 0
                and os.environ.get("TREX_LEAF_CODES", "1") != "0"):
            cb = torch.empty(int(lib().trex_tree_leaf_codes_bytes(self.n_leaf, self.L)),
                             dtype=torch.uint8, device=dev)
            status = torch.zeros(1, dtype=torch.int32, device=dev)
            check(lib().trex_tree_leaf_codes(ptr(self.S), self.n_leaf, self.L, self.Q, ptr(cb),
                                             cb.numel(), ptr(status), stream_handle(dev)))
            if int(status.item()) == 0:
                self.codes = cb
        # x3 without clipping: the GEMM operands are kept pre-split (S16, M16:
        # trex_tree_split_x3's layout) -- the ancestors' pass writes the next
        # S rows split, the surrogate writes M split, and the GEMMs stage
        # them without the split arithmetic (bitwise the x3 path;
        # TREX_PRESPLIT=0 keeps the f32 operands)
        self.presplit = (self.gemm == "x3" and clip_norm is None and self.Q == 4
                         and os.environ.get("TREX_PRESPLIT", "1") != "0")
        if self.presplit:
            self.S16 = torch.empty_like(self.S)
            self.ldm = (self.N + 31) // 32 * 32
            self.M16 = torch.zeros((self.N, self.ldm), **f32)
            check(lib().trex_tree_split_x3(ptr(self.S), self.N, self.K, self.K, 1.0,
                                           ptr(self.S16), self.K, stream_handle(dev)))

    def sequences(self, temperature=None):
        """S with its ancestor rows recomputed from the current ancestor
        logits (update_seq at ``temperature``; default: the temperature the
        next step will use) -- a fresh (N, L, Q) tensor, valid in every mode
        (``self.S``'s ancestor rows are not, in pre-split mode)."""
        T = self._s_temperature if temperature is None else float(temperature)
        if T is None:
            raise ValueError("sequences(): no step has fixed a temperature yet; pass one")
        out = self.S.clone()
        check(lib().trex_tree_update_seq(ptr(self.params["ancestors"]), self.n_anc, self.L,
                                         self.Q, T, ptr(out[self.n_leaf:]),
                                         stream_handle(self.S.device)))
        return out

    def _split_anc(self, st):
        """S16's ancestor rows from S's (after update_seq rewrote them)."""
        check(lib().trex_tree_split_x3(ptr(self.S[self.n_leaf:]), self.n_anc, self.K, self.K, 1.0,
                                       ptr(self.S16[self.n_leaf:]), self.K, st))

    def _gram(self, st):
        N, K = self.N, self.K
        if self.presplit and self.codes is not None:
            # exact one-hot leaf rows: their zero lo plane's products skipped
            check(lib().trex_tree_gram_skip_x3p_codes(
                ptr(self.S16), N, K, self.skip_rows, 1.0, ptr(self.codes), self.codes.numel(),
                self.n_leaf, self.Q, ptr(self.G), ptr(self.ws), self.ws.numel(), st))
        elif self.presplit:
            check(lib().trex_tree_gram_skip_x3p(ptr(self.S16), N, K, self.skip_rows, 1.0,
                                                ptr(self.G), ptr(self.ws), self.ws.numel(), st))
        elif self.gemm == "x3":
            check(lib().trex_tree_gram_skip_x3(ptr(self.S), N, K, self.skip_rows, 1.0,
                                               ptr(self.G), ptr(self.ws), self.ws.numel(), st))
        else:
            check(lib().trex_tree_gram_skip(ptr(self.S), N, K, self.skip_rows, ptr(self.G),
                                            ptr(self.ws), self.ws.numel(), st))

    def _combine(self, st, grad_scale, state):
        """surrogate loss / dA / M (and M16), graph constraint, one reduce."""
        check(lib().trex_tree_surrogate_constraint(
            ptr(self.A), ptr(self.G), self.N, self.scale, grad_scale, state, ptr(self.loss),
            ptr(self.dA), ptr(self.M), float(self.N + 1),
            ptr(self.M16) if self.presplit else None, self.ldm if self.presplit else 0,
            ptr(self.ws), st))

    def _mf(self, st):
        """d loss / dS for the ancestor rows only (leaf rows are fixed data)."""
        L_ = lib()
        N, K = self.N, self.K
        dS = self.dS[self.n_leaf:]
        if self.presplit:
            cb = self.codes
            check(L_.trex_tree_mf_rows_x3p(ptr(self.M16), self.ldm, ptr(self.S16), N, K,
                                           self.n_leaf, self.n_anc, float(N + 1), 1.0,
                                           ptr(cb) if cb is not None else None,
                                           cb.numel() if cb is not None else 0, self.n_leaf,
                                           self.Q, ptr(dS), st))
        elif self.codes is not None:
            check(L_.trex_tree_mf_rows_x3_codes(ptr(self.M), ptr(self.S), N, K, self.n_leaf,
                                                self.n_anc, float(N + 1), 1.0, ptr(self.codes),
                                                self.codes.numel(), self.n_leaf, self.Q, ptr(dS),
                                                st))
        elif self.gemm == "x3":
            check(L_.trex_tree_mf_rows_x3(ptr(self.M), ptr(self.S), N, K, self.n_leaf, self.n_anc,
                                          float(N + 1), 1.0, ptr(dS), st))
        else:
            check(L_.trex_tree_mf_rows(ptr(self.M), ptr(self.S), N, K, self.n_leaf, self.n_anc,
                                       ptr(dS), st))

    def step(self, temperature: float, noise, next_temperature=None):
        """One optimisation step; returns the (device) loss before the update.

        ``next_temperature``: the temperature the following ``step`` will be
        called with (default: the same).  Without clipping the Adam kernel
        then also writes that step's S rows (update_seq folded into the
        update, ``trex_adam_seq_update_step``); a following call with a
        different temperature recomputes them, so the hint only affects
        speed, never results."""
        L_ = lib()
        st = stream_handle(self.S.device)
        T = float(temperature)
        p = self.params
        N = self.N
        if self._s_temperature != T:
            check(L_.trex_tree_update_seq(ptr(p["ancestors"]), self.n_anc, self.L, self.Q, T,
                                          ptr(self.S[self.n_leaf:]), st))
            if self.presplit:
                self._split_anc(st)
        self._s_temperature = None
        check(L_.trex_tree_update_tree(ptr(p["tree_params"]), ptr(noise), None, N, self.n_anc,
                                       1.0, ptr(self.A), st))
        self._gram(st)
        if self.reducer is not None:
            self.reducer(self.G[self.g_row0:])
            check(L_.trex_tree_gram_mirror(ptr(self.G), N, self.g_row0, st))
        # surrogate loss / dA / M, then the graph constraint (loss and dA
        # accumulated), one reduce for both
        self._combine(st, T, None)
        self._mf(st)
        if self.opt.clip is None:
            o = self.opt
            o.count += 1
            # the device step record catches up lazily (Adam.sync_state)
            o._state_stale = True
            # update_tree's VJP with the tree_params' Adam step in one pass
            check(L_.trex_tree_update_tree_bwd_adam(
                ptr(self.A), ptr(self.dA), None, N, self.n_anc, 1.0,
                ptr(self.grads["tree_params"]), ptr(p["tree_params"]),
                ptr(o.mu["tree_params"]), ptr(o.nu["tree_params"]), o.count, None,
                float(o.lr), float(o.b1), float(o.b2), float(o.eps), st))
            # update_seq VJP fused into the ancestors' Adam update (the logits
            # gradient never round-trips through HBM); bitwise the same as
            # update_seq_bwd + Adam.step
            # ... and update_seq of the next step folded in (S rows rewritten
            # in place from the new logits)
            Tn = T if next_temperature is None else float(next_temperature)
            if self.presplit:
                check(L_.trex_adam_seq_update_step_x3p(
                    ptr(self.dS[self.n_leaf:]), self.n_anc, self.L, self.Q, T, Tn,
                    ptr(p["ancestors"]), ptr(o.mu["ancestors"]), ptr(o.nu["ancestors"]), o.count,
                    float(o.lr), float(o.b1), float(o.b2), float(o.eps), None, 1.0,
                    ptr(self.S16[self.n_leaf:]), st))
            else:
                check(L_.trex_adam_seq_update_step(
                    ptr(self.dS[self.n_leaf:]), self.n_anc, self.L, self.Q, T, Tn,
                    ptr(p["ancestors"]), ptr(o.mu["ancestors"]), ptr(o.nu["ancestors"]), o.count,
                    float(o.lr), float(o.b1), float(o.b2), float(o.eps),
                    ptr(self.S[self.n_leaf:]), st))
            self._s_temperature = Tn
        else:
            check(L_.trex_tree_update_tree_bwd(ptr(self.A), ptr(self.dA), None, N, self.n_anc,
                                               1.0, ptr(self.grads["tree_params"]), st))
            check(L_.trex_tree_update_seq_bwd(ptr(self.S[self.n_leaf:]),
                                              ptr(self.dS[self.n_leaf:]), self.n_anc, self.L,
                                              self.Q, T, ptr(self.grads["ancestors"]), st))
            self.opt.step(self.params, self.grads)
        return self.loss

    # ------------------------------------------------------------------
    # checkpoint / resume (the C5 loop's params + Adam state)
    # ------------------------------------------------------------------
    def state_dict(self) -> dict:
        """Host copies of everything a resumed loop needs: tree_params,
        ancestor logits and the Adam state (count, mu, nu).  S, G and the
        other buffers are recomputed from them."""
        return {"params": {k: v.detach().cpu().clone() for k, v in self.params.items()},
                "opt": self.opt.state_dict()}

    def load_state_dict(self, sd: dict):
        for k, v in sd["params"].items():
            if k not in self.params or tuple(self.params[k].shape) != tuple(v.shape):
                raise ValueError(f"TreeOptimizer.load_state_dict: params[{k!r}] does not match")
            self.params[k].copy_(v.to(self.params[k].device, dtype=self.params[k].dtype))
        self.opt.load_state_dict(sd["opt"])
        self._s_temperature = None  # the next step recomputes the ancestor rows of S

    def save_checkpoint(self, path):
        """``np.savez`` of ``state_dict`` (flat keys, no pickled objects)."""
        sd = self.state_dict()
        flat = {"count": np.asarray(sd["opt"]["count"], dtype=np.int64)}
        for k, v in sd["params"].items():
            flat[f"params/{k}"] = v.numpy()
        for name in ("mu", "nu"):
            for k, v in sd["opt"][name].items():
                flat[f"{name}/{k}"] = v.numpy()
        np.savez(path, **flat)

    def load_checkpoint(self, path):
        """Resume from ``save_checkpoint`` output (``np.load`` without pickle)."""
        torch = _torch()
        with np.load(path, allow_pickle=False) as z:
            sd = {"params": {}, "opt": {"count": int(z["count"]), "mu": {}, "nu": {}}}
            for key in z.files:
                if "/" not in key:
                    continue
                group, name = key.split("/", 1)
                t = torch.from_numpy(np.array(z[key]))
                if group == "params":
                    sd["params"][name] = t
                else:
                    sd["opt"][group][name] = t
        self.load_state_dict(sd)

    # ------------------------------------------------------------------
    # device loop (graph-capturable step)
    # ------------------------------------------------------------------
    def device_loop(self, temperatures, noise_seed: int, *, capture: bool = True):
        """The optimisation loop with everything per-step on the device --
        the reference's jitted train_step loop (tests/test_convergence.py:
        238-261; lax.fori_loop in src/trex/evals/benchmark.py:167-200):
        step k (1-based, continuing this optimiser's count) anneals at
        temperatures[k - 1] (the next step's temperature is temperatures[k],
        for update_seq folded into the Adam pass) and draws its Gumbel noise
        from trex_gumbel_noise(noise_seed, k).  With ``capture`` one step is
        captured in a hipGraph and replayed; otherwise the same launches run
        eagerly.  Bitwise the same as ``step(temperatures[k - 1],
        gumbel_noise_step(noise_seed, k, ...), temperatures[k])``.  Needs
        no clipping and no process group (the sharded Gram all-reduce is a
        host collective)."""
        return _TreeDeviceLoop(self, temperatures, noise_seed, capture)


class _TreeDeviceLoop:
    def __init__(self, opt: TreeOptimizer, temperatures, noise_seed: int, capture: bool):
        torch = _torch()
        if opt.opt.clip is not None or opt.group is not None:
            raise ValueError("device_loop: clip_norm / site sharding are host-driven; use step()")
        self.opt = opt
        dev = opt.S.device
        self.temps = torch.as_tensor(temperatures, dtype=torch.float32).to(dev).contiguous()
        self.n_temps = self.temps.numel()
        self.host_temps = [float(t) for t in self.temps.cpu()]
        self.seed = int(noise_seed) & (2**64 - 1)
        self.noise = torch.empty((opt.N - 1, opt.n_anc), dtype=torch.float32, device=dev)
        self.graph = None
        opt.opt.sync_state()
        k0 = opt.opt.count  # steps taken so far
        if k0 >= self.n_temps:
            raise ValueError("temperatures must cover the next step")
        self._refresh_rows()
        if capture:
            # capture records launches without running them: the state
            # advances only on replays
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._launch()

    def _refresh_rows(self):
        """The ancestor rows of S (S16 when pre-split) at the next step's
        temperature.  A captured step reads them as the previous replay left
        them, so anything that replaced them in between -- load_state_dict /
        load_checkpoint, an eager step() with another next temperature --
        must be caught up eagerly before the next replay."""
        o = self.opt
        T = self.host_temps[o.opt.count]
        if o._s_temperature != T:
            st = stream_handle(o.S.device)
            check(lib().trex_tree_update_seq(ptr(o.params["ancestors"]), o.n_anc, o.L, o.Q, T,
                                             ptr(o.S[o.n_leaf:]), st))
            if o.presplit:
                o._split_anc(st)
            o._s_temperature = T

    def _launch(self):
        o = self.opt
        L_ = lib()
        st = stream_handle(o.S.device)
        p = o.params
        N = o.N
        a = o.opt
        state = ptr(a.state)
        check(L_.trex_step_advance(state, float(a.b1), float(a.b2), ptr(self.temps), self.n_temps,
                                   st))
        check(L_.trex_gumbel_noise(self.seed, state, self.noise.numel(), ptr(self.noise), st))
        check(L_.trex_tree_update_tree(ptr(p["tree_params"]), ptr(self.noise), None, N, o.n_anc,
                                       1.0, ptr(o.A), st))
        o._gram(st)
        o._combine(st, 0.0, state)
        dS = o.dS[o.n_leaf:]
        o._mf(st)
        check(L_.trex_tree_update_tree_bwd_adam(
            ptr(o.A), ptr(o.dA), None, N, o.n_anc, 1.0, ptr(o.grads["tree_params"]),
            ptr(p["tree_params"]), ptr(a.mu["tree_params"]), ptr(a.nu["tree_params"]), 0, state,
            float(a.lr), float(a.b1), float(a.b2), float(a.eps), st))
        if o.presplit:
            check(L_.trex_adam_seq_update_step_x3p(
                ptr(dS), o.n_anc, o.L, o.Q, 1.0, 1.0, ptr(p["ancestors"]),
                ptr(a.mu["ancestors"]), ptr(a.nu["ancestors"]), 0, float(a.lr), float(a.b1),
                float(a.b2), float(a.eps), state, 1.0, ptr(o.S16[o.n_leaf:]), st))
        else:
            check(L_.trex_adam_seq_update_step_dev(ptr(dS), o.n_anc, o.L, o.Q, state,
                                                   ptr(p["ancestors"]), ptr(a.mu["ancestors"]),
                                                   ptr(a.nu["ancestors"]), float(a.lr),
                                                   float(a.b1), float(a.b2), float(a.eps),
                                                   ptr(o.S[o.n_leaf:]), st))

    def run(self, n_steps: int):
        """n_steps steps (graph replays or eager launches); returns the
        (device) loss of the last one."""
        o = self.opt
        if o.opt.count + n_steps > self.n_temps:
            raise ValueError("the temperature schedule does not cover these steps")
        o.opt.sync_state()  # eager steps since the capture counted on the host
        if n_steps > 0:
            self._refresh_rows()
        for _ in range(int(n_steps)):
            if self.graph is not None:
                self.graph.replay()
            else:
                self._launch()
            o.opt.count += 1
        o._s_temperature = self.host_temps[min(o.opt.count, self.n_temps - 1)]
        return o.loss
