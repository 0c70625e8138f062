"""Id dictionary for Java Long vertex ids (gcc_idmap_*, host-only C++ in libgelly_cc.so): dense ids in first-seen
order, and canonical labels = the minimum ORIGINAL id of each component in signed Long order — the reference's
DisjointSet<Long> (…/summaries/DisjointSet.java:30-34) keys its HashMap by the id itself. No GPU needed."""
import numpy as np
import pytest

from gelly_stream import GellyCCError, IdDictionary


def python_components(pairs):
    """Reference restatement over original ids: a plain dict union-find, canonical = min id per component."""
    parent = {}

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for a, b in pairs:
        for x in (a, b):
            parent.setdefault(x, x)
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)
    return {v: find(v) for v in parent}


def test_first_seen_order_and_lookup():
    d = IdDictionary(16)
    ids = [7, -3, 1 << 40, 7, -(1 << 62), 0, -3]
    assert d.map(ids).tolist() == [0, 1, 2, 0, 3, 4, 1]
    assert len(d) == 5
    assert d.ids().tolist() == [7, -3, 1 << 40, -(1 << 62), 0]
    assert d.lookup(1 << 40) == 2 and d.lookup(12345) is None
    assert d.map(np.array([[0, 99]], dtype=np.int64)).tolist() == [[4, 5]]
    d.close()


def test_overflowing_batch_maps_nothing():
    """a batch whose new ids do not all fit is rejected whole: no id of it gets a dense id (a caller that
    retries or drops the batch must not find mapped ids that were never folded), and the table stays consistent."""
    d = IdDictionary(10)
    assert d.map(list(range(100, 108))).tolist() == list(range(8))
    with pytest.raises(GellyCCError):
        d.map([100, 5, 6, 101, 7])  # three new ids, room for two
    assert len(d) == 8
    assert all(d.lookup(x) is None for x in (5, 6, 7))
    assert all(d.lookup(100 + i) == i for i in range(8))
    assert d.map([6, 104, 5]).tolist() == [8, 4, 9]  # the same ids fit once the batch does
    assert d.ids().tolist() == list(range(100, 108)) + [6, 5]
    d.close()


def test_capacity_is_enforced():
    d = IdDictionary(3)
    d.map([1, 2, 3, 1, 2])
    with pytest.raises(GellyCCError):
        d.map([4])
    with pytest.raises(GellyCCError):
        IdDictionary(0)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_canonical_labels_are_min_original_ids(seed):
    """Random graph over ids spread across the whole Long range (negative and > 2^32): any representative labelling
    of the dense forest maps to min-original-id labels, equal to a union-find over the original ids."""
    rng = np.random.default_rng(seed)
    universe = rng.integers(-(1 << 63), (1 << 63) - 1, size=300, dtype=np.int64)
    pairs = universe[rng.integers(0, universe.size, size=(220, 2))]
    want = python_components(pairs.tolist())
    d = IdDictionary(1000)
    dense = d.map(pairs)
    # dense forest labels with an arbitrary representative per component (max dense id here, not min)
    comp = python_components(dense.tolist())
    members = {}
    for v, r in comp.items():
        members.setdefault(r, []).append(v)
    lab = np.full(len(d) + 5, 0xFFFFFFFF, dtype=np.uint32)
    for ms in members.values():
        lab[ms] = max(ms)
    got = d.canonical(lab[:len(d)])
    ids = d.ids()
    assert {int(ids[i]): int(got[i]) for i in range(len(d))} == want
    # ids the forest has not seen get the `unseen` value
    lab2 = lab[:len(d)].copy()
    lab2[0] = 0xFFFFFFFF
    assert d.canonical(lab2, unseen=-1)[0] == -1


def test_canonical_rejects_out_of_range_labels():
    d = IdDictionary(8)
    d.map([10, 20])
    with pytest.raises(GellyCCError):
        d.canonical(np.array([0, 5], dtype=np.uint32))
