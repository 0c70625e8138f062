// gelly/ConnectedComponents.hpp — C++ host mirror of …/library/ConnectedComponents.java on an MI355X.
//
//   ConnectedComponents(long mergeWindowTime)  ConnectedComponents.java:52-54
//       = SummaryBulkAggregation(new UpdateCC(), new CombineCC(), new DisjointSet<K>(), mergeWindowTime, false)
//   UpdateCC.foldEdges                          :83-86   ds.union(vertex, vertex2); return ds
//   CombineCC.reduce                            :116-125 merge the smaller forest into the larger
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

#include "gelly/Aggregation.hpp"
#include "gelly/DisjointSet.hpp"

namespace gelly {

template <typename K, typename EV = NullValue>
class UpdateCC : public EdgesFold<K, EV, DisjointSet<K>> {
   public:
    DisjointSet<K> foldEdges(DisjointSet<K> ds, K vertex, K vertex2, EV) override {
        ds.union_(vertex, vertex2);
        return ds;
    }
    // the whole window batch of one partition in one device fold (edge values are ignored, as in the reference)
    DisjointSet<K> foldEdgeBatch(DisjointSet<K> ds, const Edge<K, EV>* edges, size_t n) override {
        std::vector<uint32_t> pairs(2 * n);
        for (size_t i = 0; i < n; ++i) {
            pairs[2 * i] = checked(ds, edges[i].src);
            pairs[2 * i + 1] = checked(ds, edges[i].trg);
        }
        ds.fold(pairs.data(), n);
        return ds;
    }

   private:
    static uint32_t checked(const DisjointSet<K>& ds, K v) {
        if (v < 0 || (uint64_t)v >= ds.idCapacity())
            throw GellyException(GCC_E_INVALID, "vertex id " + std::to_string((long long)v) + " out of range");
        return (uint32_t)v;
    }
};

template <typename K>
class CombineCC : public ReduceFunction<DisjointSet<K>> {
   public:
    DisjointSet<K> reduce(DisjointSet<K> s1, DisjointSet<K> s2) override {
        const uint64_t count1 = s1.getMatches().size();
        const uint64_t count2 = s2.getMatches().size();
        if (count1 <= count2) {
            s2.merge(s1);
            return s2;
        }
        s1.merge(s2);
        return s1;
    }
};

template <typename K, typename EV = NullValue>
class ConnectedComponents : public SummaryBulkAggregation<K, EV, DisjointSet<K>, DisjointSet<K>> {
   public:
    using Base = SummaryBulkAggregation<K, EV, DisjointSet<K>, DisjointSet<K>>;
    // id_capacity / device: the u32 id range and GPU of the device summary (the reference's HashMap grows)
    ConnectedComponents(int64_t mergeWindowTime, uint32_t id_capacity, int device = 0)
        : Base(std::make_shared<UpdateCC<K, EV>>(), std::make_shared<CombineCC<K>>(),
               [id_capacity, device] { return DisjointSet<K>(id_capacity, device); }, mergeWindowTime, false) {}

    // Fused form of SummaryBulkAggregation.run for CC: with transientState=false the running summary after
    // window w has the partition of summary ∪ edges(w), so each window is folded straight into the running
    // device forest (all partitions at once) and the summary object itself is emitted, like the reference's
    // Merger collects the same summary object every window.
    void run(const SimpleEdgeStream<K, EV>& stream, const typename Base::Emit& emit) override {
        std::optional<DisjointSet<K>> summary;
        for (auto [b, e] : stream.windows(this->timeMillis())) {
            if (!summary) summary = this->getInitialValue();
            summary = this->getUpdateFun()->foldEdgeBatch(*summary, stream.edges().data() + b, e - b);
            emit(*summary);
        }
    }
};

}  // namespace gelly
