"""Generate tests/golden fixtures (run from the repo root).

The reference (JAX) cannot be imported in this image, so the fixtures are:
  * kat_sankoff.json -- hand-derived known answers on the reference's own test
    fixtures (tests/test_sankoff.py:9-72; derivation in SURVEY.md §4) and the
    tie-averaged gradient derived by hand for the same tree;
  * sankoff_cases.npz -- oracle outputs on seeded inputs, pinned so later
    oracle edits cannot drift silently (tests/test_oracle.py re-derives them).

    python tests/golden/make_golden.py
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from _cases import int_cost, random_leaves, random_topologies, weird_children  # noqa: E402
from oracle.sankoff_ref import run_sankoff_ref  # noqa: E402
from oracle.softmin_ref import batched_fwd_bwd_ref  # noqa: E402
from trex_amd.topology import adjacency_from_children  # noqa: E402

KAT = {
    "source": "reference tests/test_sankoff.py:39-72 fixture; values hand-derived",
    "adjacency_edges": [[0, 3], [1, 3], [2, 4], [3, 4]],
    "cost": [[0, 1], [1, 0]],
    "leaf_sequences": [[0, 1], [1, 0], [0, 0]],
    "n_all": 5, "n_states": 2, "n_leaves": 3,
    "total": 2.0,
    "dp": [[[0, 1e5], [1e5, 0], [0, 1e5], [1, 1], [1, 2]],
           [[1e5, 0], [0, 1e5], [0, 1e5], [1, 1], [1, 2]]],
    "reconstructed": [[0, 1], [1, 0], [0, 0], [0, 0], [0, 0]],
    # d total / d cost (tie-averaged, hard): root argmin state 0 at both
    # sites; every message picks a unique argmin; see DESIGN.md "KAT".
    "d_cost": [[6, 2], [0, 0]],
    "run_dp_fixture": {
        "source": "reference tests/test_sankoff.py:9-36",
        "adjacency": [[0, 1, 0], [0, 1, 0], [0, 0, 0]],
        "sequences": [[0], [1], [0]],
        "dp": [[0, 1e5], [1e5, 0], [2e5, 2e5]],
        "bt_row2": [[-1, 0, -1, 0], [-1, 1, -1, 1]],
    },
}


def cases():
    out = {}
    k = 0
    for n, L, Q in [(8, 37, 4), (16, 64, 3), (12, 50, 2)]:
        ch = random_topologies(2, n, seed=10 + k)
        leaves = random_leaves(2, n, L, Q, seed=20 + k, missing=0.05)
        cost = int_cost(Q, seed=30 + k)
        out[f"c{k}"] = (ch, leaves, cost)
        k += 1
    for case in ("fwdref", "dag"):
        ch = weird_children(case)[None]
        leaves = random_leaves(1, 8, 40, 4, seed=40 + k)
        out[case] = (ch, leaves, int_cost(4, seed=50 + k))
        k += 1
    return out


def compute(ch, leaves, cost):
    res = {}
    hard = batched_fwd_bwd_ref(ch, leaves, cost, 0.0)
    soft = batched_fwd_bwd_ref(ch, leaves, cost, 0.5)
    res["hard_dp"] = hard["dp"].astype(np.float32)
    res["hard_tree_score"] = hard["tree_score"]
    res["hard_d_cost"] = hard["d_cost"]
    res["soft_tree_score"] = soft["tree_score"]
    res["soft_d_cost"] = soft["d_cost"]
    adj = adjacency_from_children(ch)
    n_all = ch.shape[1]
    nl = (n_all + 1) // 2
    recon = []
    for b in range(ch.shape[0]):
        r = run_sankoff_ref(adj[b], cost, leaves[b].astype(np.float32), n_all, cost.shape[0],
                            nl, return_path=True)
        recon.append(r[0])
    res["recon"] = np.stack(recon)
    return res


def main():
    with open(os.path.join(HERE, "kat_sankoff.json"), "w") as f:
        json.dump(KAT, f, indent=1)
    arrays = {}
    for name, (ch, leaves, cost) in cases().items():
        arrays[f"{name}/children"] = ch
        arrays[f"{name}/leaves"] = leaves
        arrays[f"{name}/cost"] = cost
        for key, val in compute(ch, leaves, cost).items():
            arrays[f"{name}/{key}"] = val
    np.savez_compressed(os.path.join(HERE, "sankoff_cases.npz"), **arrays)
    print("wrote", sorted(set(k.split("/")[0] for k in arrays)))


if __name__ == "__main__":
    main()
