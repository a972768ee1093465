"""trex_amd.tree.PRNGKey / split: host-side key handling (no GPU)."""

from __future__ import annotations

from trex_amd.tree import PRNGKey, split


def test_split_is_deterministic_and_distinct():
    k = PRNGKey(7)
    a, b = split(k)
    assert (a, b) == split(PRNGKey(7))
    assert len({k, a, b}) == 3
    assert len(set(split(k, 5))) == 5
    assert split(k, 5)[:2] == (a, b)  # child i does not depend on num
    assert PRNGKey(2**64 + 7) == k  # 64-bit seeds
