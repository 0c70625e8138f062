// Host replay of the CC forest's device code (gelly-streaming_amd/csrc/uf_device.h): the exact per-edge and per-id
// functions the gfx950 kernels run, executed by host threads, kernel by kernel, under a model of gfx950's
// in-kernel memory behaviour, and checked after every window against a sequential union-find.
// Test infrastructure (tests/test_uf_replay.py drives it; the oracle pins the sequential labels).
//
// Memory model of one kernel (uf_device.h ReplayHooks): every memory operation is a scheduling point; a plain load
// returns, with probability stale/1000, an older value of the word from the history SINCE THE KERNEL STARTED
// (its value at the kernel boundary, or any value stored or swapped in since) — what a load served from a CU's
// non-coherent L1, or another XCD's L2, may return. Atomics (CAS, atomicMin, atomicOr) act on the fresh value,
// as gfx950's memory-side atomics do. Kernel boundaries make atomics visible (stream order: release/acquire), but
// NOT every plain store (round 4, measured on the MI355X: tools/stress_inc.py): with probability
// late/1000 a plain store also LANDS AGAIN at a random point of the next kernel (controlled scheduler) or at its end
// (free threads), overwriting whatever that kernel wrote to the word — a store still on its way when the kernel ended.
//
// Two schedulers:
//   controlled ("ctl"): the threads run one memory operation at a time, the next thread chosen at random at every
//     operation (a randomised interleaving explorer), stale values drawn from the whole in-kernel history;
//     small forests, many seeds;
//   free ("free"): real concurrent threads (ASan / TSan builds), stale = the word's kernel-start value; big forests.
//
// Pipelines (each is the kernel sequence of one product path, gelly_cc.hip):
//   out            fold_kernel + compress_kernel (out of place: labels into the spare buffer;     [product]
//                  read-only finds since round 5 — argument "split" restores round 4's splitting compress)
//   inplace_split  fold + a compress IN PLACE with path splitting (round 1's first compress)      [removed]
//   inplace_nosplit fold + a compress in place, read-only finds                                  [experiment]
//   inc            fold_kernel<REC> (bloom, no path splitting: UFRec) + compress_inc_kernel<true> [product]
//                  in place (inc_inplace), its labels stored write-through (round 5: gcc::st_through)
//   inc_split      path splitting in the recording fold and plain label stores in the in-place     [removed]
//                  compress (round 3's product: the late split store over the compress's root is the stale label)
//   filter         fold_filtered_kernel's round: atomicMin hook + one-round-late settle + ring   [product]
//                  entries (unite_entry), then the compress
//   absorb         a peer's merge message: msg_absorb_bits_kernel (plain store of new ids) then  [product]
//                  msg_absorb_kernel (lists), then the compress
//   init           a fresh forest's seeded / bucketed start: parent[] := C ? g : UNSEEN by plain   [product]
//                  stores (bucket_init_kernel, seed_pack_kernel<true>), then the filtered fold, then the compress
//   pipe           the pipelined emission (round 5): window 0 as "out", then per window the recording fold  [product]
//                  with touched marks (fold_pipe_kernel) and, in the SAME kernel on other threads, the scan of
//                  the previous window (compress_pipe_kernel: labels, new-id words, the bloom ring), then the
//                  window's resolve (pipe_resolve_kernel); each emission checked after its scan
//   pipe_allhit    pipe with every label a bloom hit (maximal false positives: the roots snapshot of untouched
//                  labels, UNSEEN or stale by parity, decides)
//
// Input on stdin: V W then W window sizes, then the edges "u v". Args: pipeline mode threads seeds stale_pm [late_pm
// [late_depth [any|plain [split|ro]]]]: late stores up to late_depth kernels late, landing over any later write or
// only over later plain stores, and the full compress's finds splitting paths or read-only.
// Output: one line per seed with the failing windows, then "pipeline=<p> runs=<n> bad_runs=<k> bad_windows=<m>"
// and, on the first failure, the id, its label, the expected label and the parent chain. With mode "labels" the
// sequential reference labels of the last window are printed (one per line) for the oracle cross-check.
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "uf_device.h"

using gcc::u32;
using gcc::u64;
static constexpr u32 U = GCC_UNSEEN_DEV;

static u64 splitmix(u64& s) {
    u64 z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ---------------------------------------------------------------------------------------------------------------
// the scheduler and the memory model
// ---------------------------------------------------------------------------------------------------------------
static thread_local int t_tid = -1;
static thread_local u64 t_rng = 1;

struct Sched {
    std::mutex m;
    std::condition_variable cv;
    int turn = -1;
    std::vector<char> alive;
    u64 rng = 1;
    u64 ops = 0, budget = 0;

    void pick_locked() {
        int n = 0;
        for (char a : alive) n += a;
        if (!n) {
            turn = -1;
            return;
        }
        int k = (int)(splitmix(rng) % (u64)n);
        for (int i = 0; i < (int)alive.size(); ++i)
            if (alive[i] && k-- == 0) {
                turn = i;
                return;
            }
    }
    void yield() {
        std::unique_lock<std::mutex> lk(m);
        if (++ops > budget) {
            std::fprintf(stderr, "livelock: %llu memory operations in one kernel\n", (unsigned long long)ops);
            std::fflush(stderr);
            std::_Exit(3);
        }
        pick_locked();
        cv.notify_all();
        cv.wait(lk, [&] { return turn == t_tid; });
    }
    void enter() {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return turn == t_tid; });
    }
    void leave() {
        std::unique_lock<std::mutex> lk(m);
        alive[t_tid] = 0;
        pick_locked();
        cv.notify_all();
    }
};

struct Model : gcc::ReplayHooks {
    bool controlled = false;
    unsigned stale_pm = 0;
    unsigned late_pm = 0;
    // late plain stores (round 5): a store issued in kernel k lands again during kernel k + d,
    // d drawn from 1..late_depth (2 covers the out-of-place compress's buffer swap: the buffer a kernel stored into is
    // written again two kernels later). late_any: a late store may land over ANY later write of the word; otherwise
    // ("plain" flavour) only over later PLAIN stores — a memory-side atomic of a later kernel is ordered after it (the
    // pattern the MI355X showed: tools/stress_inc.py, a plain split store over the in-place compress's plain store)
    unsigned late_depth = 1;
    bool late_any = true;
    Sched sched;
    struct Late {
        u32* p;
        u32 v;
        u64 at;      // op index in the kernel it lands in (controlled), ~0: at that kernel's end
        u64 issued;  // global op index when it was stored
        unsigned k_left;
    };
    std::mutex late_m;
    std::vector<Late> pending, landing;
    u64 kernel_ops = 0;
    std::atomic<u64> gops{0};
    u64 n_late = 0, n_dropped = 0;
    // the tracked words: every parent[] array of the pipeline (loads elsewhere are never stale)
    std::vector<std::pair<u32*, u32>> arrays;
    std::vector<std::vector<std::vector<u32>>> hist;  // [array][id] -> values since the kernel start (ctl)
    std::vector<std::vector<u32>> start;              // [array][id] -> value at the kernel start (free)
    std::vector<std::vector<u64>> last_atomic;        // [array][id] -> global op of the last atomic write

    void reset_run() {
        pending.clear();
        landing.clear();
        last_atomic.assign(arrays.size(), {});
        for (size_t a = 0; a < arrays.size(); ++a) last_atomic[a].assign(arrays[a].second, 0);
    }
    bool locate(const u32* p, size_t& a, size_t& i) const {
        for (a = 0; a < arrays.size(); ++a)
            if (p >= arrays[a].first && p < arrays[a].first + arrays[a].second) {
                i = (size_t)(p - arrays[a].first);
                return true;
            }
        return false;
    }
    void land(const Late& l) {
        size_t a, i;
        if (!locate(l.p, a, i)) return;
        if (!late_any && __atomic_load_n(&last_atomic[a][i], __ATOMIC_RELAXED) > l.issued) {
            ++n_dropped;  // an atomic wrote the word after this store was issued: ordered after it
            return;
        }
        __atomic_store_n(l.p, l.v, __ATOMIC_RELAXED);
        if (controlled) hist[a][i].push_back(l.v);
    }
    void kernel_begin() {
        landing.clear();
        std::vector<Late> keep;
        for (auto& l : pending) {
            if (--l.k_left == 0) {
                l.at = controlled ? splitmix(sched.rng) % 4096 : ~0ull;
                landing.push_back(l);
            } else {
                keep.push_back(l);
            }
        }
        pending.swap(keep);
        kernel_ops = 0;
        hist.resize(arrays.size());
        start.resize(arrays.size());
        for (size_t a = 0; a < arrays.size(); ++a) {
            const u32* b = arrays[a].first;
            const u32 n = arrays[a].second;
            if (controlled) {
                hist[a].assign(n, {});
                for (u32 i = 0; i < n; ++i) hist[a][i].push_back(b[i]);
            } else {
                start[a].assign(b, b + n);
            }
        }
    }
    void before(const u32*) override {
        gops.fetch_add(1, std::memory_order_relaxed);
        if (controlled) {
            sched.yield();
            ++kernel_ops;  // serialised by the scheduler
            for (auto& l : landing)
                if (l.at == kernel_ops) land(l);
        }
    }
    void stored(u32* p, u32 v) override {
        if (!late_pm || (splitmix(t_rng) % 1000) >= late_pm) return;
        size_t a, i;
        if (!locate(p, a, i)) return;
        const unsigned d = 1 + (unsigned)(splitmix(t_rng) % (late_depth ? late_depth : 1));
        std::lock_guard<std::mutex> g(late_m);
        pending.push_back({p, v, 0, gops.load(std::memory_order_relaxed), d});
        ++n_late;
    }
    void atomic(const u32* p) override {
        size_t a, i;
        if (locate(p, a, i)) __atomic_store_n(&last_atomic[a][i], gops.load(std::memory_order_relaxed), __ATOMIC_RELAXED);
    }
    // the end of a kernel: the late stores due in it that have not landed yet land now
    void kernel_end() {
        for (auto& l : landing)
            if (l.at > kernel_ops) land(l);
        landing.clear();
    }
    u32 load(const u32* p, u32 fresh) override {
        if (!stale_pm || (splitmix(t_rng) % 1000) >= stale_pm) return fresh;
        size_t a, i;
        if (!locate(p, a, i)) return fresh;
        if (!controlled) return start[a][i];
        const auto& h = hist[a][i];
        return h[(size_t)(splitmix(t_rng) % h.size())];
    }
    void wrote(const u32* p, u32 v) override {
        size_t a, i;
        if (controlled && locate(p, a, i)) hist[a][i].push_back(v);  // serialised by the scheduler
    }

    // One kernel: T threads, thread t runs body(t); a kernel boundary on both sides.
    void kernel(int T, u64 seed, const std::function<void(int)>& body) {
        kernel_begin();
        std::vector<std::thread> th;
        if (controlled) {
            sched.alive.assign(T, 1);
            sched.rng = seed;
            sched.ops = 0;
            {
                std::unique_lock<std::mutex> lk(sched.m);
                sched.turn = -2;  // nobody runs until every thread exists
            }
        }
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                t_tid = t;
                t_rng = seed * 1000003ull + (u64)t * 7919ull + 1;
                if (controlled) sched.enter();
                body(t);
                if (controlled) sched.leave();
            });
        if (controlled) {
            std::unique_lock<std::mutex> lk(sched.m);
            sched.pick_locked();
            sched.cv.notify_all();
        }
        for (auto& x : th) x.join();
        kernel_end();
    }
};

static Model g_model;

// how often the paths under test were taken (summed over runs; printed with the verdict)
static std::atomic<u64> n_hooks{0}, n_hook_unions{0}, n_absorb_stores{0}, n_inc_finds{0};

// ---------------------------------------------------------------------------------------------------------------
// the sequential reference (min-id roots) and helpers
// ---------------------------------------------------------------------------------------------------------------
struct SeqUF {
    std::vector<u32> p;
    explicit SeqUF(u32 V) : p(V, U) {}
    u32 find(u32 x) {
        while (p[x] != x) x = p[x];
        return x;
    }
    void unite(u32 a, u32 b) {
        if (p[a] == U) p[a] = a;
        if (p[b] == U) p[b] = b;
        a = find(a);
        b = find(b);
        if (a < b) p[b] = a;
        else if (b < a) p[a] = b;
    }
    std::vector<u32> labels() {
        std::vector<u32> l(p.size(), U);
        for (u32 v = 0; v < p.size(); ++v)
            if (p[v] != U) l[v] = find(v);
        return l;
    }
};

// the component holding most ids (any component is a correct tracked set; the vote only picks a useful one)
static u32 giant_of(const std::vector<u32>& lab) {
    std::vector<u32> cnt(lab.size(), 0);
    u32 best = U, bc = 0;
    for (u32 l : lab)
        if (l != U && ++cnt[l] > bc) {
            bc = cnt[l];
            best = l;
        }
    return best;
}

struct Edge {
    u32 a, b;
};

// ---------------------------------------------------------------------------------------------------------------
// the kernels (bodies as in gelly_cc.hip: grid-stride over items, thread t takes items t, t+T, ...)
// ---------------------------------------------------------------------------------------------------------------
struct Forest {
    u32 V;
    std::vector<u32> parent, spare;
    std::vector<u32> bloom[2];
    int bloom_cur = 0;
    bool rec_all = false;
    // the pipelined emission: labels in `spare`; roots and new-id words by window parity, blooms in a ring of 3,
    // touched marks (hooked | new, two words per 32 ids)
    u32 nw32;
    std::vector<u32> roots[2], born[2], touched, pbloom[3];
    Forest(u32 v) : V(v), parent(v, U), spare(v, U), nw32((v + 31) / 32) {
        bloom[0].assign(gcc::kBloomBits / 32, 0);
        bloom[1].assign(gcc::kBloomBits / 32, 0);
        for (int i = 0; i < 2; ++i) {
            roots[i].assign(v, U);
            born[i].assign(nw32, 0);
        }
        touched.assign(2 * (size_t)nw32, 0);
        for (int i = 0; i < 3; ++i) pbloom[i].assign(gcc::kBloomBits / 32, 0);
    }
};

// rec: 0 plain fold; 1 the recording fold (UFRec: no path splitting, the product); 2 recording with path splitting
static void k_fold(Forest& f, const Edge* e, u64 n, int T, u64 seed, int rec) {
    u32* par = f.parent.data();
    u32* bl = f.bloom[f.bloom_cur].data();
    g_model.kernel(T, seed, [&](int t) {
        gcc::NoCount c;
        for (u64 i = (u64)t; i < n; i += (u64)T) {
            if (rec == 1) gcc::UFRec::unite(par, e[i].a, e[i].b, c, gcc::BloomRec{bl});
            else if (rec == 2) gcc::UF::unite(par, e[i].a, e[i].b, c, gcc::BloomRec{bl});
            else gcc::UF::unite(par, e[i].a, e[i].b, c);
        }
    });
}

// compress_bits_kernel: labels into the spare buffer (plain stores, through the late-store model), then swap. SPLIT:
// its finds split paths in the old buffer (plain stores there too; round 4's product), else read-only finds (round 5)
template <bool SPLIT>
static void k_compress_out(Forest& f, int T, u64 seed) {
    u32* par = f.parent.data();
    u32* lab = f.spare.data();
    const u32 V = f.V;
    g_model.kernel(T, seed, [&](int t) {
        gcc::NoCount c;
        for (u32 v = (u32)t; v < V; v += (u32)T) {
            const u32 p = gcc::ld(&par[v]);
            const u32 l = p >= v ? p : gcc::UnionFind<gcc::LoadPlain, SPLIT>::find_from(par, v, p, c);
            gcc::st(&lab[v], l);
        }
    });
    std::swap(f.parent, f.spare);
    f.rec_all = false;
}
static bool g_compress_split = false;  // the product's full compress: split (round 4) or read-only finds (round 5)
static void k_compress_out(Forest& f, int T, u64 seed) {
    if (g_compress_split) k_compress_out<true>(f, T, seed);
    else k_compress_out<false>(f, T, seed);
}

// bucket_init_kernel / seed_pack_kernel<true>: parent[v] := v in C ? g : UNSEEN with plain stores (the reset and
// every union inside C in one write); the filtered / bucketed passes then hook with memory-side atomics
static void k_init(Forest& f, const std::vector<char>& inC, u32 g, int T, u64 seed) {
    u32* par = f.parent.data();
    const u32 V = f.V;
    g_model.kernel(T, seed, [&](int t) {
        for (u32 v = (u32)t; v < V; v += (u32)T) gcc::st(&par[v], inC[v] ? g : U);
    });
    f.rec_all = false;
}

// the in-place compress variants: each slot written only by its own thread, with the root
template <bool SPLIT>
static void k_compress_inplace(Forest& f, int T, u64 seed) {
    u32* par = f.parent.data();
    const u32 V = f.V;
    g_model.kernel(T, seed, [&](int t) {
        gcc::NoCount c;
        for (u32 v = (u32)t; v < V; v += (u32)T) {
            const u32 p = gcc::ld(&par[v]);
            if (p >= v) continue;
            const u32 r = gcc::UnionFind<gcc::LoadPlain, SPLIT>::find_from(par, v, p, c);
            if (r != p) gcc::st(&par[v], r);
        }
    });
    f.rec_all = false;
}

// compress_inc_kernel<true>: the bloom is the kernel's LDS copy (taken at its start); 4 consecutive ids per lane
// read before any of them is labelled (the 16-B load), only changed slots written; the other bloom is cleared.
// through: the labels written write-through (gcc::st_through, round 5's product) or with plain stores (rounds 3-4)
static void k_compress_inc_inplace(Forest& f, int T, u64 seed, bool through) {
    u32* par = f.parent.data();
    const std::vector<u32> lds = f.bloom[f.bloom_cur];
    const u32 V = f.V;
    const u32 chunks = (V + 3) / 4;
    g_model.kernel(T, seed, [&](int t) {
        for (u32 ch = (u32)t; ch < chunks; ch += (u32)T) {
            u32 p[4], lab[4];
            const u32 v0 = ch * 4;
            for (u32 k = 0; k < 4; ++k) p[k] = (v0 + k < V) ? gcc::ld(&par[v0 + k]) : U;
            for (u32 k = 0; k < 4; ++k)
                if (v0 + k < V) {
                    if (p[k] < v0 + k && gcc::bloom_test(lds.data(), p[k]))
                        n_inc_finds.fetch_add(1, std::memory_order_relaxed);
                    lab[k] = gcc::inc_label(par, lds.data(), v0 + k, p[k]);
                    if (lab[k] != p[k]) {
                        if (through) gcc::st_through(&par[v0 + k], lab[k]);
                        else gcc::st(&par[v0 + k], lab[k]);
                    }
                }
        }
    });
    std::fill(f.bloom[f.bloom_cur ^ 1].begin(), f.bloom[f.bloom_cur ^ 1].end(), 0u);
}

// the product's compress_now: incremental in place when every mutation since the last compress was recorded
static void compress_product_inc(Forest& f, int T, u64 seed, bool through = true) {
    if (f.rec_all) {
        k_compress_inc_inplace(f, T, seed, through);
    } else {
        k_compress_out(f, T, seed);
        std::fill(f.bloom[f.bloom_cur ^ 1].begin(), f.bloom[f.bloom_cur ^ 1].end(), 0u);
    }
    f.bloom_cur ^= 1;
    f.rec_all = true;
}

// The pipelined emission in one kernel: threads [0, T) run fold_pipe_kernel over window w's edges (bloom w % 3 and
// the touched marks), threads [T, 2T) — when w >= 1 — compress_pipe_kernel for window w-1 (its bloom as the kernel's
// LDS copy, its roots / new-id words of parity (w-1) % 2, clearing the bloom that window w+1 will record into): the
// product runs them on two streams, so any interleaving of the two is possible. A scan thread takes 32-id words:
// every id of the word labelled (gcc::pipe_label), then the word cleared.
static void k_fold_scan(Forest& f, const Edge* e, u64 n, u32 w, int T, u64 seed, bool allhit) {
    u32* par = f.parent.data();
    u32* lab = f.spare.data();
    u32* bl = f.pbloom[w % 3].data();
    const bool scan = w >= 1;
    const u32 sw = w - 1, p = sw & 1;
    std::vector<u32> lds = scan ? f.pbloom[sw % 3] : std::vector<u32>();
    if (allhit) std::fill(lds.begin(), lds.end(), ~0u);
    u32* clear = f.pbloom[(sw + 2) % 3].data();
    const u32 V = f.V, nw = f.nw32;
    g_model.kernel(scan ? 2 * T : T, seed, [&](int t) {
        if (t < T) {
            gcc::NoCount c;
            for (u64 i = (u64)t; i < n; i += (u64)T)
                gcc::UFRec::unite(par, e[i].a, e[i].b, c, gcc::PipeRec{bl, f.touched.data()});
            return;
        }
        const u32 s = (u32)(t - T);
        for (u32 k = s; k < nw; k += (u32)T) {
            const u32 bw = gcc::ld(&f.born[p][k]);
            for (u32 b = 0; b < 32 && k * 32 + b < V; ++b) {
                const u32 v = k * 32 + b;
                const u32 l = gcc::ld(&lab[v]);
                const u32 r = gcc::pipe_label(lds.data(), f.roots[p].data(), v, l, (bw >> b) & 1u);
                if (r != l) {
                    gcc::st_through(&lab[v], r);
                    gcc::amin(&par[v], r);  // the forest follows the labels (concurrently with the fold's threads)
                }
            }
            if (bw) gcc::st_through(&f.born[p][k], 0u);
        }
        for (size_t k = s; k < f.pbloom[0].size(); k += (size_t)T) __atomic_store_n(&clear[k], 0u, __ATOMIC_RELAXED);
    });
}

// pipe_resolve_kernel for window w: per 32-id word, the touched marks taken and cleared (the product: one 64-bit
// atomic exchange), the new ids' word written out, every touched id's root snapshot
static void k_resolve(Forest& f, u32 w, int T, u64 seed) {
    u32* par = f.parent.data();
    const u32 p = w & 1, nw = f.nw32;
    g_model.kernel(T, seed, [&](int t) {
        for (u32 k = (u32)t; k < nw; k += (u32)T) {
            const u32 hk = __atomic_exchange_n(&f.touched[2 * (size_t)k], 0u, __ATOMIC_RELAXED);
            const u32 nb = __atomic_exchange_n(&f.touched[2 * (size_t)k + 1], 0u, __ATOMIC_RELAXED);
            if (nb) gcc::st_through(&f.born[p][k], nb);
            for (u32 m = hk | nb; m; m &= m - 1) {
                const u32 x = k * 32 + (u32)__builtin_ctz(m);
                gcc::st_through(&f.roots[p][x], gcc::pipe_root(par, x));
            }
        }
    });
}

// fold_filtered_kernel<HOOK>'s edge handling per thread: rounds of N edges; in a round the bitmap lookups, then the
// atomicMin hooks of (T, id > g) edges, then the PREVIOUS round's hooks settled (a hook whose old value shows that
// the id hung elsewhere pushes (g, old) to the ring), then the round's slow edges pushed; the ring drained (up to
// 64 entries, here `drain` ones) whenever `drain` are pending, and at the end; ring entries by unite_entry.
static void k_filtered(Forest& f, const Edge* e, u64 n, const std::vector<char>& inT, u32 g, int T, u64 seed,
                       int N, u32 drain) {
    u32* par = f.parent.data();
    g_model.kernel(T, seed, [&](int t) {
        std::vector<Edge> ring;
        size_t wd = 0;
        struct Carry {
            u32 other, old;
            bool hook;
        };
        std::vector<Carry> carry, cur;
        auto push = [&](u32 a, u32 b) {
            ring.push_back({a, b});
            if (ring.size() - wd >= drain) {
                const size_t end = std::min(ring.size(), wd + 64);
                for (; wd < end; ++wd) gcc::unite_entry(par, ring[wd].a, ring[wd].b, g);
            }
        };
        auto settle = [&](std::vector<Carry>& cs) {
            for (auto& c : cs)
                if (c.hook && gcc::hook_needs_union(c.old, c.other, g)) {
                    n_hook_unions.fetch_add(1, std::memory_order_relaxed);
                    push(g, c.old);
                }
            cs.clear();
        };
        // this thread's edges: items t, t+T, ... taken N at a time
        std::vector<u64> mine;
        for (u64 i = (u64)t; i < n; i += (u64)T) mine.push_back(i);
        for (size_t r0 = 0; r0 < mine.size(); r0 += (size_t)N) {
            const size_t r1 = std::min(mine.size(), r0 + (size_t)N);
            std::vector<Edge> slow;
            cur.clear();
            for (size_t k = r0; k < r1; ++k) {
                const Edge x = e[mine[k]];
                const bool ia = inT[x.a], ib = inT[x.b];
                const u32 other = ia ? x.b : x.a;
                const bool hook = (ia != ib) && other > g;
                if (hook) {
                    n_hooks.fetch_add(1, std::memory_order_relaxed);
                    cur.push_back({other, gcc::hook_min(par, other, g), true});
                }
                else if (!(ia && ib)) slow.push_back({ia ? g : x.a, ib ? g : x.b});
            }
            settle(carry);
            for (auto& s : slow) push(s.a, s.b);
            carry.swap(cur);
        }
        settle(carry);
        for (; wd < ring.size(); ++wd) gcc::unite_entry(par, ring[wd].a, ring[wd].b, g);
    });
    f.rec_all = false;
}

// msg_absorb_bits_kernel: ids of the peer's giant outside T joined to R (absorb_join); one id per item
static void k_absorb_bits(Forest& f, const std::vector<u32>& ids, u32 R, int T, u64 seed) {
    u32* par = f.parent.data();
    g_model.kernel(T, seed, [&](int t) {
        for (size_t i = (size_t)t; i < ids.size(); i += (size_t)T) {
            if (ids[i] > R && __atomic_load_n(&par[ids[i]], __ATOMIC_RELAXED) == U)
                n_absorb_stores.fetch_add(1, std::memory_order_relaxed);
            gcc::absorb_join(par, ids[i], R);
        }
    });
    f.rec_all = false;
}

// msg_absorb_kernel: the lone giant (no overlap with T) against its own root, then the (v, label) list
static void k_absorb_lists(Forest& f, const std::vector<Edge>& pairs, int T, u64 seed) {
    u32* par = f.parent.data();
    g_model.kernel(T, seed, [&](int t) {
        gcc::NoCount c;
        for (size_t i = (size_t)t; i < pairs.size(); i += (size_t)T) gcc::UF::unite(par, pairs[i].a, pairs[i].b, c);
    });
    f.rec_all = false;
}

// ---------------------------------------------------------------------------------------------------------------
// one run of a pipeline over the windows
// ---------------------------------------------------------------------------------------------------------------
struct Failure {
    u32 window = 0, id = 0, got = 0, want = 0;
    std::vector<u32> chain;
};

static void chain_of(const std::vector<u32>& par, u32 v, std::vector<u32>& out) {
    out.clear();
    for (int k = 0; k < 16 && v != U; ++k) {
        out.push_back(v);
        const u32 p = par[v];
        if (p == v || p == U) break;
        v = p;
    }
}

static int run(const std::string& pipe, u32 V, const std::vector<u64>& wstart, const std::vector<Edge>& E, int T,
               u64 seed, std::vector<u32>& bad_windows, Failure& first) {
    Forest f(V);
    SeqUF ref(V), peer(V);
    g_model.arrays = {{f.parent.data(), V}, {f.spare.data(), V}, {f.roots[0].data(), V}, {f.roots[1].data(), V},
                      {f.born[0].data(), f.nw32}, {f.born[1].data(), f.nw32}};
    std::vector<u32> want_prev;  // pipe: the previous window's labels, checked after its scan
    int bad = 0;
    auto check = [&](const std::vector<u32>& got, const std::vector<u32>& want, u32 win) {
        for (u32 v = 0; v < V; ++v)
            if (got[v] != want[v]) {
                if (!bad++) {
                    first.window = win;
                    first.id = v;
                    first.got = got[v];
                    first.want = want[v];
                    chain_of(f.parent, v, first.chain);
                }
                bad_windows.push_back(win);
                return;
            }
    };
    // forest invariant (every pipeline): a seen id points at a seen id no larger than itself
    auto invariant = [&](u32 win) {
        for (u32 v = 0; v < V; ++v) {
            const u32 p = f.parent[v];
            if (p != U && (p > v || f.parent[p] == U)) {
                std::fprintf(stderr, "invariant broken: window %u id %u parent %u\n", win, v, p);
                std::exit(2);
            }
        }
    };
    g_model.reset_run();  // late stores of an earlier run point into its freed forest
    std::vector<char> inT(V, 0);
    u32 g = U;
    const u32 W = (u32)wstart.size() - 1;
    for (u32 w = 0; w < W; ++w) {
        const Edge* e = E.data() + wstart[w];
        const u64 n = wstart[w + 1] - wstart[w];
        const u64 ks = seed * 131 + w * 17;
        for (u64 i = 0; i < n; ++i) ref.unite(e[i].a, e[i].b);
        if (pipe == "out") {
            k_fold(f, e, n, T, ks + 1, false);
            k_compress_out(f, T, ks + 2);
        } else if (pipe == "inplace_split") {
            k_fold(f, e, n, T, ks + 1, false);
            k_compress_inplace<true>(f, T, ks + 2);
        } else if (pipe == "inplace_nosplit") {
            k_fold(f, e, n, T, ks + 1, false);
            k_compress_inplace<false>(f, T, ks + 2);
        } else if (pipe == "inc" || pipe == "inc_split") {
            // inc_split is round 3's product as it was: the recording fold with path splitting AND plain label stores
            // in the in-place compress
            k_fold(f, e, n, T, ks + 1, pipe == "inc" ? 1 : 2);
            compress_product_inc(f, T, ks + 2, pipe == "inc");
        } else if (pipe == "init") {
            // a fresh forest's seeded / bucketed start: C = the component of the window's most frequent endpoint
            // among its own edges (any set inside one component of the batch is a valid seed), g = min C, one plain
            // store per id, then the filtered fold against C; later windows as "filter"
            if (g == U) {
                SeqUF s(V);
                std::vector<u32> deg(V, 0);
                for (u64 i = 0; i < n; ++i) s.unite(e[i].a, e[i].b), ++deg[e[i].a], ++deg[e[i].b];
                u32 h = 0;
                for (u32 v = 1; v < V; ++v)
                    if (deg[v] > deg[h]) h = v;
                const u32 rh = s.find(h);
                g = U;
                for (u32 v = 0; v < V; ++v) {
                    inT[v] = s.p[v] != U && s.find(v) == rh;
                    if (inT[v] && g == U) g = v;
                }
                k_init(f, inT, g, T, ks + 1);
            }
            k_filtered(f, e, n, inT, g, T, ks + 3, 2, 2);
            k_compress_out(f, T, ks + 2);
            g = giant_of(f.parent);
            for (u32 v = 0; v < V; ++v) inT[v] = g != U && f.parent[v] == g;
        } else if (pipe == "filter") {
            if (g == U) k_fold(f, e, n, T, ks + 1, false);  // the first window: nothing tracked yet
            else k_filtered(f, e, n, inT, g, T, ks + 1, 2, 2);
            k_compress_out(f, T, ks + 2);
            g = giant_of(f.parent);
            for (u32 v = 0; v < V; ++v) inT[v] = g != U && f.parent[v] == g;
        } else if (pipe == "absorb") {
            // this forest folds the window's first half; a peer (sequential) the second half; then the peer's
            // merge message is absorbed: bitmap of its giant + (v, label) list of its other seen ids
            const u64 h = n / 2;
            k_fold(f, e, h, T, ks + 1, false);
            k_compress_out(f, T, ks + 2);
            for (u64 i = h; i < n; ++i) peer.unite(e[i].a, e[i].b);
            const std::vector<u32> pl = peer.labels();
            const u32 gp = giant_of(pl);
            const u32 R = giant_of(f.parent);
            bool overlap = false;
            for (u32 v = 0; v < V && R != U && gp != U; ++v) overlap |= pl[v] == gp && f.parent[v] == R;
            std::vector<u32> ids;
            std::vector<Edge> pairs;
            for (u32 v = 0; v < V; ++v) {
                if (pl[v] == U) continue;
                if (pl[v] == gp) {
                    if (overlap) {
                        if (f.parent[v] != R && v != R) ids.push_back(v);  // U \ T
                    } else if (v != gp) {
                        pairs.push_back({v, gp});
                    }
                } else {
                    pairs.push_back({v, pl[v]});
                }
            }
            if (overlap) k_absorb_bits(f, ids, R, T, ks + 3);
            k_absorb_lists(f, pairs, T, ks + 4);
            k_compress_out(f, T, ks + 5);
        } else if (pipe == "pipe" || pipe == "pipe_allhit") {
            if (w == 0) {  // a fresh forest: fold + full compress; then the mode starts (labels = a copy of parent[])
                k_fold(f, e, n, T, ks + 1, false);
                k_compress_out(f, T, ks + 2);
                check(f.parent, ref.labels(), w);
                // the mode starts (pipe_enter): the forest is copied (a blit: plain stores) into the other buffer and
                // goes on there; the labels stay in the compress's buffer and become L
                u32* src = f.parent.data();
                u32* dst = f.spare.data();
                g_model.kernel(T, ks + 4, [&](int t) {
                    for (u32 v = (u32)t; v < V; v += (u32)T) gcc::st(&dst[v], src[v]);
                });
                std::swap(f.parent, f.spare);
            } else {
                k_fold_scan(f, e, n, w, T, ks + 1, pipe == "pipe_allhit");  // + the scan of window w-1
                if (w >= 2) check(f.spare, want_prev, w - 1);
                k_resolve(f, w, T, ks + 2);
            }
            want_prev = ref.labels();
            if (w + 1 == W && w >= 1) {  // the last window's scan alone
                k_fold_scan(f, nullptr, 0, w + 1, T, ks + 3, pipe == "pipe_allhit");
                check(f.spare, want_prev, w);
            }
            invariant(w);
            continue;
        } else {
            std::fprintf(stderr, "unknown pipeline %s\n", pipe.c_str());
            std::exit(1);
        }
        // the emission is read after the compress (the product's consumer reads after a synchronisation)
        // after the compress parent[] IS the label array (out of place: swapped in; in place: rewritten)
        check(f.parent, ref.labels(), w);
        invariant(w);
    }
    return bad;
}

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s pipeline ctl|free|labels threads seeds stale_pm < stream\n", argv[0]);
        return 1;
    }
    const std::string pipe = argv[1], mode = argv[2];
    const int T = std::atoi(argv[3]);
    const int seeds = std::atoi(argv[4]);
    g_model.stale_pm = (unsigned)std::atoi(argv[5]);
    g_model.late_pm = argc > 6 ? (unsigned)std::atoi(argv[6]) : 0;
    g_model.late_depth = argc > 7 ? (unsigned)std::atoi(argv[7]) : 1;
    g_model.late_any = argc > 8 ? std::string(argv[8]) != "plain" : true;
    g_compress_split = argc > 9 ? std::string(argv[9]) == "split" : false;
    u32 V, W;
    if (std::scanf("%u %u", &V, &W) != 2) return 1;
    std::vector<u64> ws(W + 1, 0);
    for (u32 i = 0; i < W; ++i) {
        unsigned long long s;
        if (std::scanf("%llu", &s) != 1) return 1;
        ws[i + 1] = ws[i] + s;
    }
    std::vector<Edge> E(ws[W]);
    for (auto& e : E)
        if (std::scanf("%u %u", &e.a, &e.b) != 2 || e.a >= V || e.b >= V) return 1;
    if (mode == "labels") {  // the sequential reference of the whole stream (checked against the oracle)
        SeqUF ref(V);
        for (auto& e : E) ref.unite(e.a, e.b);
        for (u32 l : ref.labels()) std::printf("%u\n", l);
        return 0;
    }
    g_model.controlled = mode == "ctl";
    g_model.sched.budget = 4000000;
    gcc::replay = &g_model;
    int bad_runs = 0;
    u64 bad_windows = 0;
    Failure first;
    bool have_first = false;
    for (int s = 0; s < seeds; ++s) {
        std::vector<u32> bw;
        Failure fl;
        const int b = run(pipe, V, ws, E, T, 0x5EED0000ull + (u64)s, bw, fl);
        if (b) {
            ++bad_runs;
            bad_windows += (u64)b;
            if (!have_first) {
                first = fl;
                have_first = true;
                std::printf("seed %d: first bad window %u: id %u label %u want %u chain", s, fl.window, fl.id, fl.got,
                            fl.want);
                for (u32 x : fl.chain) std::printf(" %u", x);
                std::printf("\n");
            }
        }
    }
    gcc::replay = nullptr;
    std::printf("pipeline=%s mode=%s threads=%d runs=%d bad_runs=%d bad_windows=%llu hooks=%llu hook_unions=%llu "
                "absorb_stores=%llu inc_finds=%llu late_stores=%llu late_dropped=%llu\n",
                pipe.c_str(), mode.c_str(), T, seeds, bad_runs, (unsigned long long)bad_windows,
                (unsigned long long)n_hooks.load(), (unsigned long long)n_hook_unions.load(),
                (unsigned long long)n_absorb_stores.load(), (unsigned long long)n_inc_finds.load(),
                (unsigned long long)g_model.n_late, (unsigned long long)g_model.n_dropped);
    return 0;
}
