"""GPU: the reference-literal Candidates (csrc/gelly_literal.hip, gcc_literal_*) against the reference's own output.

The signed forest (test_gpu_bipartite.py) is BipartitenessCheck with the intended semantics. LiteralCandidates
reproduces Candidates.merge as written (…/summaries/Candidates.java:77-192): the KAT lines of BipartitenessCheckTest /
NonBipartitnessCheckTest verbatim, and on every window of every bip_*.json fixture the (success, toString) that the
literal restatement recorded (tests/golden/make_golden_bip.py, "reference_literal") — including the windows where the
reference is not a partition join (overlapping components, a missed odd cycle): those are reproduced, not pinned.
"""
import glob
import os

import numpy as np
import pytest

from gelly_stream import LiteralBipartitenessCheck, LiteralCandidates, SimpleEdgeStream

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_reference_kats_verbatim(golden):
    fx = golden("bip_kat.json")
    for key in ("bipartite", "non_bipartite"):
        k = fx[key]
        stream = SimpleEdgeStream(np.array(k["edges"], dtype=np.uint32))
        out = [c.toString() for c in stream.aggregate(LiteralBipartitenessCheck(500, id_capacity=k["V"]))]
        assert out == [k["expected"]], key


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "bip_*.json"))))
def test_fixture_windows_reproduce_the_reference(path, golden):
    """Every window's emitted summary (the SummaryBulkAggregation topology: per-partition partials, combined in
    order, then the Merger) equals the reference's line."""
    name = os.path.basename(path)
    if name == "bip_kat.json":
        return
    fx = golden(name)
    pairs = np.array(fx["pairs"], dtype=np.uint32)
    starts = fx["window_starts"]
    ts = np.zeros(len(pairs), dtype=np.int64)
    for w in range(len(starts) - 1):
        ts[starts[w]:starts[w + 1]] = w * 1000
    stream = SimpleEdgeStream(pairs, timestamps=ts, parallelism=fx["partitions"])
    want = [w for w in fx["windows"] if w is not None]
    got = [(c.getSuccess(), c.toString()) for c in stream.aggregate(LiteralBipartitenessCheck(1000, id_capacity=fx["V"]))]
    assert len(got) == len(want)
    diverging = 0
    for w, (g, x) in enumerate(zip(got, want)):
        lit = x["reference_literal"]
        assert g == (lit["success"], lit["string"]), (name, w)
        diverging += not x["reference_literal_agrees"]
    if name in ("bip_random_bipartite.json", "bip_large_bipartite_p4.json", "bip_same_vertex_sets_p2.json"):
        assert diverging, "the fixture exercises a window where the reference is not a partition join"


def test_identical_vertex_sets_are_skipped():
    """Candidates.java:91-95: two summaries over {1, 2, 3} (paths 1-2-3 and 1-3-2) merge into a triangle, which the
    reference does not check (the components are skipped): success stays true."""
    a, b = LiteralCandidates(8), LiteralCandidates(8)
    a.fold(np.array([[1, 2], [2, 3]], dtype=np.uint32))
    b.fold(np.array([[1, 3], [3, 2]], dtype=np.uint32))
    assert a.toString() == "(true,{1={1=(1,true), 2=(2,false), 3=(3,true)}})"
    assert a.merge(b).getSuccess()
    assert a.toString() == "(true,{1={1=(1,true), 2=(2,false), 3=(3,true)}})"
    a.close()
    b.close()


def test_smaller_input_key_leaves_the_self_component():
    """Candidates.java:176-189: {5, 9} then the edge (3, 9): the input's vertices go under key 3, the component
    keyed 5 stays as it is (9 is in both)."""
    c = LiteralCandidates(16)
    c.fold(np.array([[5, 9], [3, 9]], dtype=np.uint32))
    assert c.toString() == "(true,{3={3=(3,true), 9=(9,false)}, 5={5=(5,true), 9=(9,false)}})"
    c.close()


def test_odd_cycle_fails_for_good():
    c = LiteralCandidates(8)
    c.fold(np.array([[1, 2], [2, 3], [3, 1], [4, 5]], dtype=np.uint32))
    assert not c.getSuccess() and c.toString() == "(false,{})"
    c.reset()
    assert c.getSuccess() and c.toString() == "(true,{})"
    c.close()
