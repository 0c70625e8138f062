"""CPU: the CC forest's device code (gelly-streaming_amd/csrc/uf_device.h) replayed on host threads
(tests/cpp/test_uf_replay.cpp) under a model of gfx950's in-kernel memory behaviour: every memory operation a
scheduling point, plain loads answered by stale but historically valid values (any value the word held since the
kernel started), atomics on the fresh value, kernel boundaries making atomics visible — and, since round 4, plain
stores that may land AGAIN in the next kernel (late_pm), after that kernel's own writes: measured on the MI355X
(tools/stress_inc.py: C3 in 1M-edge windows, 747 wrong windows in 7854 streams with the recording fold's path
splitting, none without it).

Each pipeline is the kernel sequence of one product path (gelly_cc.hip): the fold + out-of-place compress, the
bloom-recording fold + in-place incremental compress (inc_inplace), the filtered fold's atomicMin hook with its
one-round-late settle and ring unions, the merge absorb with its plain store of new ids, and (round 5) the pipelined
emission — the scan of window w in the same kernel as window w+1's fold, on other threads, with a bloom that answers
every label (pipe_allhit) so that the roots snapshot's UNSEEN / same-parity entries decide. All must reproduce the
sequential labels in every window, under the controlled interleaving explorer (ASan+UBSan build) and with real
concurrent threads (ASan and TSan builds). The in-place compress WITH path splitting (round 1's first compress) must
FAIL: it is the named race (a thread's split store of a grandparent into slot v lands after v's owner stored v's
root), and the harness has to be able to see it (the controlled leg without any stale load). The sequential reference is pinned to the oracle.
"""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")
ASAN = os.path.join(CPP, "build", "test_uf_replay")
TSAN = os.path.join(CPP, "build", "test_uf_replay_tsan")
PRODUCT = ["out", "inc", "filter", "absorb", "init", "pipe", "pipe_allhit"]


@pytest.fixture(scope="module")
def build():
    r = subprocess.run(["make", "-s", "-C", CPP, "build/test_uf_replay", "build/test_uf_replay_tsan"],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("building the replay failed:\n" + r.stderr[-2000:])


def stream_text(parts, V):
    text = f"{V} {len(parts)}\n" + " ".join(str(len(p)) for p in parts) + "\n"
    return text + "\n".join(f"{int(a)} {int(b)}" for p in parts for a, b in p) + "\n"


def run(exe, pipe, mode, threads, seeds, stale_pm, text, late_pm=0, late_depth=1, late_kind="plain", compress="ro",
        allow_exit=False):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", TSAN_OPTIONS="halt_on_error=1")
    p = subprocess.run([exe, pipe, mode, str(threads), str(seeds), str(stale_pm), str(late_pm), str(late_depth), late_kind,
                        compress], input=text, capture_output=True, text=True, env=env, timeout=600)
    if allow_exit and p.returncode == 2 and "invariant broken" in p.stderr:
        return 1, p.stderr  # a late store broke the forest itself (counts as a failing run)
    assert p.returncode == 0, f"{pipe} {mode}: exit {p.returncode}\n{p.stderr[-3000:]}"
    assert "ThreadSanitizer" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-3000:]
    last = p.stdout.strip().split("\n")[-1]
    kv = dict(x.split("=") for x in last.split())
    run.counts = {k: int(v) for k, v in kv.items()
                  if k in ("hooks", "hook_unions", "absorb_stores", "inc_finds", "late_stores", "late_dropped")}
    return int(kv["bad_runs"]), p.stdout


def chain_stream(seed):
    """Small stream with deep chains: descending paths (each union hooks the previous root one lower), a star,
    random edges, and a late window that joins the paths (hooks of long chains' roots)."""
    rng = np.random.default_rng(seed)
    V = 24
    w0 = [(k, k + 1) for k in range(11, -1, -1)] + [(k, k + 1) for k in range(22, 12, -1)]
    w1 = [tuple(x) for x in rng.integers(0, V, size=(6, 2))]
    w2 = [(12, 11), (23, 0)] + [(5, int(x)) for x in rng.integers(0, V, size=3)]
    return V, [np.array(w, dtype=np.int64) for w in (w0, w1, w2)]


def big_stream(seed, V=1 << 15, windows=4):
    rng = np.random.default_rng(seed)
    parts = []
    for _ in range(windows):
        r = rng.integers(0, V, size=(20000, 2))
        s = int(rng.integers(0, V - 600))
        path = np.stack([np.arange(s + 500, s, -1), np.arange(s + 501, s + 1, -1)], 1)
        h = int(rng.integers(0, V))
        star = np.stack([np.full(300, h), rng.integers(0, V, 300)], 1)
        e = np.concatenate([r, path, star])
        rng.shuffle(e)
        parts.append(e)
    return V, parts


def test_sequential_reference_matches_oracle(build):
    for V, parts in (chain_stream(1), big_stream(2, V=4096, windows=2)):
        p = subprocess.run([ASAN, "out", "labels", "1", "1", "0"], input=stream_text(parts, V), capture_output=True,
                           text=True, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"), timeout=120)
        assert p.returncode == 0, p.stderr
        got = np.array(p.stdout.split(), dtype=np.uint64).astype(np.uint32)
        pairs = np.concatenate(parts).astype(np.uint32)
        starts = [0, len(pairs)]
        want = orc.cc_stream(pairs, starts, V, want_labels=True)["labels"][-1]
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("stale_pm", [0, 150])
def test_controlled_interleavings(build, stale_pm):
    """Randomised interleaving explorer: one memory operation at a time, 3 threads, deep-chain streams."""
    jobs = [(pipe, seed) for pipe in PRODUCT + ["inplace_nosplit"] for seed in (1, 2)]

    def one(job):
        pipe, seed = job
        V, parts = chain_stream(seed)
        return pipe, seed, run(ASAN, pipe, "ctl", 3, 60, stale_pm, stream_text(parts, V))

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        for pipe, seed, (bad, out) in ex.map(one, jobs):
            assert bad == 0, f"{pipe} (stream seed {seed}, stale {stale_pm}/1000):\n{out}"


def test_split_race_is_seen(build):
    """The in-place compress with path splitting loses the race the product's out-of-place compress avoids: a
    split store parent[v] = grandparent (a non-root) lands after v's owner stored root(v). No stale load needed."""
    V, parts = chain_stream(1)
    bad, out = run(ASAN, "inplace_split", "ctl", 3, 300, 0, stream_text(parts, V))
    assert bad > 0, out
    V, parts = big_stream(5)
    bad, out = run(ASAN, "inplace_split", "free", 8, 10, 50, stream_text(parts, V))
    assert bad > 0, out


@pytest.mark.parametrize("exe", ["asan", "tsan"])
def test_free_threads(build, exe):
    """Real concurrent threads on a 32K-id stream (random edges, descending paths, stars), stale loads injected."""
    V, parts = big_stream(3)
    text = stream_text(parts, V)
    binary = ASAN if exe == "asan" else TSAN
    exercised = {"inc": "inc_finds", "filter": "hook_unions", "absorb": "absorb_stores"}
    for pipe in PRODUCT + ["inplace_nosplit"]:
        bad, out = run(binary, pipe, "free", 8, 3 if exe == "asan" else 2, 50, text)
        assert bad == 0, f"{pipe}:\n{out}"
        if pipe in exercised:  # the path under test was taken (bloom-hit finds, hook re-unions, plain stores)
            assert run.counts[exercised[pipe]] > 0, out


def test_late_plain_stores(build):
    """Round 4's stale label, replayed, and the model round 5 closes: a plain store may
    land again up to TWO kernels late — the out-of-place compress swaps its buffers, so the buffer a kernel stores into
    is written again two kernels later — over any later PLAIN store of the word. Every plain store of parent[] and of the
    label buffers goes through the model: the folds' path splitting (UF), the compress's label stores, the in-place
    compress's, the seeded start's reset (bucket_init / seed_pack: the "init" pipeline). Memory-side atomics and
    write-through (sc1) stores are never late, and a late plain store does not land over them (the "plain" flavour:
    the compress -> fold hand-off, plain label stores then CAS hooks on the same words, runs in every window on the
    MI355X with 0 failures in 10,371 + 7,000 stress streams; tools/probe_late_store.hip 0 of 240).
    Under it: round 3's pipeline fails; every product pipeline (round 5: the full compress's finds read-only, the
    in-place compress's labels write-through) is exact; round 4's splitting full compress is NOT (its split stores into
    the old buffer land over that buffer's labels after the swap back)."""
    V, parts = big_stream(3)
    text = stream_text(parts, V)
    bad, out = run(ASAN, "inc_split", "free", 8, 4, 50, text, late_pm=20, late_depth=2)
    assert bad > 0 and run.counts["late_stores"] > 0, out
    for pipe in PRODUCT:
        bad, out = run(ASAN, pipe, "free", 8, 3, 50, text, late_pm=20, late_depth=2)
        assert bad == 0 and run.counts["late_stores"] > 0, f"{pipe}:\n{out}"
    bad, out = run(ASAN, "out", "free", 8, 3, 50, text, late_pm=20, late_depth=2, compress="split")
    assert bad > 0, out
    for seed in (1, 2):
        V2, parts2 = chain_stream(seed)
        for pipe in PRODUCT:
            bad, out = run(ASAN, pipe, "ctl", 3, 100, 100, stream_text(parts2, V2), late_pm=100, late_depth=2)
            assert bad == 0, f"{pipe} (stream seed {seed}):\n{out}"
        bad, out = run(ASAN, "inc_split", "ctl", 3, 100, 100, stream_text(parts2, V2), late_pm=100, late_depth=2)
        assert bad > 0, out


def test_late_stores_over_atomics_contradict_the_hardware(build):
    """The stronger flavour — a late plain store may land over a later memory-side ATOMIC too — fails every pipeline,
    including the compress -> fold hand-off that runs in every window on the MI355X without a single failure in the
    stress runs. So the measurements refute it, and the model above is the one the product is built
    to."""
    V2, parts2 = chain_stream(1)
    bad, out = run(ASAN, "out", "ctl", 3, 100, 100, stream_text(parts2, V2), late_pm=100, late_depth=1,
                   late_kind="any", allow_exit=True)
    assert bad > 0, out
