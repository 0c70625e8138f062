// C++ host mirror tests: the reference's own tests replayed through gelly/*.hpp -> C ABI -> HIP (needs a GPU).
//   DisjointSetTest          src/test/java/org/apache/flink/graph/streaming/util/DisjointSetTest.java:36-78
//   ConnectedComponentsTest  src/test/java/org/apache/flink/graph/streaming/example/test/ConnectedComponentsTest.java
//   ConnectedComponentsExample default data (…/example/ConnectedComponentsExample.java:78, :121-133)
// Prints one PASS/FAIL line per test; exit status = number of failures.
#include <cstdio>
#include <functional>
#include <set>
#include <string>
#include <vector>

#include "gelly/ConnectedComponents.hpp"

using namespace gelly;

static int failures = 0;
#define EXPECT(cond)                                                                        \
    do {                                                                                    \
        if (!(cond)) throw std::runtime_error(std::string("expectation failed: ") + #cond); \
    } while (0)

static void run(const char* name, const std::function<void()>& body) {
    try {
        body();
        std::printf("PASS %s\n", name);
    } catch (const std::exception& e) {
        std::printf("FAIL %s: %s\n", name, e.what());
        ++failures;
    }
}

static DisjointSet<int> setup() {  // DisjointSetTest.setup :36-41
    DisjointSet<int> ds(128);
    for (int i = 0; i < 8; i++) ds.union_(i, i + 2);
    return ds;
}

int main() {
    run("DisjointSetTest.testGetMatches", [] {  // :43-46
        auto ds = setup();
        EXPECT(ds.getMatches().size() == 10);
    });
    run("DisjointSetTest.testFind", [] {  // :48-57
        auto ds = setup();
        auto root1 = ds.find(0), root2 = ds.find(1);
        EXPECT(root1 && root2 && *root1 != *root2);
        for (int i = 0; i < 10; i++) EXPECT(ds.find(i) == ((i % 2) == 0 ? root1 : root2));
        EXPECT(!ds.find(50));  // unseen key: null
    });
    run("DisjointSetTest.testMerge", [] {  // :59-78
        auto ds = setup();
        DisjointSet<int> ds2(128);
        for (int i = 0; i < 8; i++) ds2.union_(i, i + 100);
        ds2.merge(ds);
        EXPECT(ds2.getMatches().size() == 18);
        std::set<int> treeRoots;
        for (int element : ds2.getMatches().keySet()) treeRoots.insert(*ds2.find(element));
        EXPECT(treeRoots.size() == 2);
    });
    run("DisjointSet.toString", [] {
        auto ds = setup();
        EXPECT(ds.toString() == "{0=[0, 2, 4, 6, 8], 1=[1, 3, 5, 7, 9]}");
    });
    run("ConnectedComponentsTest", [] {  // 6 edges, ConnectedComponents(5) :29-38, :81; expected :19-21
        std::vector<Edge<long, NullValue>> edges = {{1, 2, {}}, {1, 3, {}}, {2, 3, {}}, {1, 5, {}}, {6, 7, {}}, {8, 9, {}}};
        SimpleEdgeStream<long, NullValue> stream(edges, (uint64_t)0);
        ConnectedComponents<long> cc(5, 10);
        std::vector<std::string> out;
        stream.aggregate(cc, [&](const DisjointSet<long>& s) { out.push_back(s.toString()); });
        EXPECT(!out.empty());
        EXPECT(out.back() == "{1=[1, 2, 3, 5], 6=[6, 7], 8=[8, 9]}");  // 3 components (:73)
    });
    run("ConnectedComponentsExample.defaultData", [] {  // 100 edges (k, k+2), ts 100k, 1000 ms windows
        std::vector<Edge<long, NullValue>> edges;
        std::vector<int64_t> ts;
        for (long k = 1; k <= 100; ++k) {
            edges.push_back({k, k + 2, {}});
            ts.push_back(k * 100);
        }
        SimpleEdgeStream<long, NullValue> stream(edges, ts);
        ConnectedComponents<long> cc(1000, 103);
        int w = 0;
        stream.aggregate(cc, [&](const DisjointSet<long>& s) {
            const long hi = std::min(102L, 10L * w + 11);
            const auto& lab = s.labels();
            for (long v = 0; v < 103; ++v) {
                const uint32_t want = (v >= 1 && v <= hi) ? (v % 2 ? 1u : 2u) : GCC_UNSEEN;
                EXPECT(lab[v] == want);
            }
            ++w;
        });
        EXPECT(w == 11);
    });
    run("SummaryBulkAggregation.genericTopologyEqualsFused", [] {
        // the reference topology (3 partitions folded into fresh partials, CombineCC, Merger) vs the fused CC run
        std::vector<Edge<long, NullValue>> edges;
        uint64_t x = 12345;
        for (int i = 0; i < 20000; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            edges.push_back({(long)((x >> 33) % 5000), (long)((x >> 13) % 5000), {}});
        }
        SimpleEdgeStream<long, NullValue> stream(edges, (uint64_t)3000, 3);
        SummaryBulkAggregation<long, NullValue, DisjointSet<long>, DisjointSet<long>> generic(
            std::make_shared<UpdateCC<long>>(), std::make_shared<CombineCC<long>>(),
            [] { return DisjointSet<long>(5000); }, 1000, false);
        ConnectedComponents<long> fused(1000, 5000);
        std::vector<std::vector<uint32_t>> a, b;
        stream.aggregate(generic, [&](const DisjointSet<long>& s) { a.push_back(s.labels()); });
        stream.aggregate(fused, [&](const DisjointSet<long>& s) { b.push_back(s.labels()); });
        EXPECT(a.size() == 7 && a == b);
    });
    run("Merger.transientState", [] {
        struct Count : ReduceFunction<DisjointSet<int>> {
            DisjointSet<int> reduce(DisjointSet<int> s1, DisjointSet<int> s2) override { s2.merge(s1); return s2; }
        } comb;
        Merger<DisjointSet<int>> keep([] { return DisjointSet<int>(16); }, &comb, false);
        Merger<DisjointSet<int>> reset([] { return DisjointSet<int>(16); }, &comb, true);
        DisjointSet<int> w1(16), w2(16);
        w1.union_(1, 2);
        w2.union_(3, 4);
        keep.flatMap(w1);
        EXPECT(keep.flatMap(w2).getMatches().size() == 4);  // running summary accumulates
        reset.flatMap(w1);
        EXPECT(reset.flatMap(w2).getMatches().size() == 2);  // transientState: summary reset after each window
    });
    run("Merger.snapshotRestore", [] {
        DisjointSet<int> ds(64);
        for (int i = 0; i < 30; ++i) ds.union_(i, (i * 7) % 64);
        DisjointSet<int> back(64);
        back.restorePairs(ds.snapshotPairs());
        EXPECT(back.labels() == ds.labels());
    });
    run("DisjointSet.outOfRangeThrows", [] {
        DisjointSet<int> ds(8);
        bool threw = false;
        try {
            ds.union_(1, 9);
        } catch (const GellyException& e) {
            threw = e.code() == GCC_E_INVALID;
        }
        EXPECT(threw);
    });
    std::printf("%d failure(s)\n", failures);
    return failures;
}
