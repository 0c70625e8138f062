"""CPU: the signed union-find the gfx950 kernels run (gelly-streaming_amd/csrc/signed_uf.h), replayed on host
threads with real atomics (tests/cpp/test_signed_uf.cpp, ASan build), against the oracle's canonical words.

The stale-read legs inject what a load served from a non-coherent L1 line may return on gfx950 (an UNSEEN the
word held once): the walks must stop at a true ancestor and the retries must reload fresh words, so the verdict
and the canonical words may not change. This is the host witness for the concurrency argument in gelly_bip.hip.
"""
import os
import subprocess

import numpy as np
import pytest

import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")
EXE = os.path.join(CPP, "build", "test_signed_uf")


@pytest.fixture(scope="module")
def replay():
    r = subprocess.run(["make", "-s", "-C", CPP, "build/test_signed_uf"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("building the signed replay failed:\n" + r.stderr[-2000:])

    def run(pairs, starts, V, threads=8, stale_pm=0):
        sizes = np.diff(np.asarray(starts, dtype=np.int64))
        text = f"{V} {threads} {len(sizes)}\n" + " ".join(map(str, sizes.tolist())) + "\n"
        text += "\n".join(f"{int(u)} {int(v)}" for u, v in pairs) + "\n"
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
        p = subprocess.run([EXE, str(stale_pm)], input=text, capture_output=True, text=True, env=env, timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        lines = p.stdout.split("\n")
        return lines[0] == "fail 1", np.array(lines[1:1 + V], dtype=np.uint64).astype(np.uint32)

    return run


def random_stream(V, E, seed, bipartite=True):
    rng = np.random.default_rng(seed)
    if not bipartite:
        return rng.integers(0, V, (E, 2)).astype(np.uint32)
    side = rng.integers(0, 2, V)
    A, B = np.flatnonzero(side == 0), np.flatnonzero(side == 1)
    e = np.stack([rng.choice(A, E), rng.choice(B, E)], axis=1).astype(np.uint32)
    flip = rng.integers(0, 2, E).astype(bool)
    e[flip] = e[flip][:, ::-1]
    return e


@pytest.mark.parametrize("stale_pm", [0, 50, 300])
def test_replay_fixture_windows(replay, golden, stale_pm):
    """bip_large_bipartite_p4 in its two windows (the stream that faulted the first device version)."""
    fx = golden("bip_large_bipartite_p4.json")
    pairs = np.array(fx["pairs"], dtype=np.uint32)
    want = orc.bip_stream(pairs, fx["window_starts"], fx["V"])
    for _ in range(5):
        failed, words = replay(pairs, fx["window_starts"], fx["V"], stale_pm=stale_pm)
        assert failed == (not want["success"][-1])
        assert np.array_equal(words, want["words"][-1])


@pytest.mark.parametrize("stale_pm", [0, 100])
@pytest.mark.parametrize("bipartite", [True, False])
def test_replay_random_vs_oracle(replay, stale_pm, bipartite):
    V, E = 4096, 20000
    pairs = random_stream(V, E, 3 + bipartite, bipartite)
    starts = [0, 500, E // 2, E]
    want = orc.bip_stream(pairs, starts, V)
    failed, words = replay(pairs, starts, V, stale_pm=stale_pm)
    assert failed == (not want["success"][-1])
    if want["success"][-1]:
        assert np.array_equal(words, want["words"][-1])
