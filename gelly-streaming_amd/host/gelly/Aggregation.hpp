// gelly/Aggregation.hpp — C++ host mirror of gelly-streaming's summary-aggregation operator surface.
//
// Reference (`…/` = src/main/java/org/apache/flink/graph/streaming/):
//   EdgesFold<K,EV,T>            …/EdgesFold.java:33-47      T foldEdges(T accum, K vertexID, K neighborID, EV edgeValue)
//   SummaryAggregation           …/SummaryAggregation.java:50-135 (+ Merger :93-135)
//   SummaryBulkAggregation       …/SummaryBulkAggregation.java:51-131
//   SimpleEdgeStream             …/SimpleEdgeStream.java:69-73, :86-90 (ctors), :100-102 (aggregate)
// Flink's runtime is not restated: windows are tumbling event-time windows of `timeMillis` over the edges'
// timestamps (or, without timestamps, the deterministic model edge i -> window i / edgesPerWindow), a window's
// edges are split into `parallelism` contiguous partitions (PartitionMapper, :93-106), and the output
// DataStream<T> becomes a callback invoked once per emitted window.
#pragma once

#include <algorithm>
#include <cstdint>
#include <functional>
#include <memory>
#include <optional>
#include <type_traits>
#include <utility>
#include <vector>

namespace gelly {

struct NullValue {};

template <typename K, typename EV>
struct Edge {  // org.apache.flink.graph.Edge<K, EV>
    K src;
    K trg;
    EV value;
};

template <typename K, typename EV, typename T>
class EdgesFold {  // …/EdgesFold.java:33-47
   public:
    virtual ~EdgesFold() = default;
    virtual T foldEdges(T accum, K vertexID, K neighborID, EV edgeValue) = 0;
    // PartialAgg.fold (:121-123) over one partition's window batch; GPU summaries override with one launch
    virtual T foldEdgeBatch(T accum, const Edge<K, EV>* edges, size_t n) {
        for (size_t i = 0; i < n; ++i) accum = foldEdges(accum, edges[i].src, edges[i].trg, edges[i].value);
        return accum;
    }
};

template <typename S>
class ReduceFunction {  // org.apache.flink.api.common.functions.ReduceFunction<S>
   public:
    virtual ~ReduceFunction() = default;
    virtual S reduce(S value1, S value2) = 0;
};

// SummaryAggregation.Merger (…/SummaryAggregation.java:93-135): the parallelism-1 running summary
template <typename S>
class Merger {
   public:
    Merger(std::function<S()> initial, ReduceFunction<S>* combiner, bool transientState)
        : initial_(std::move(initial)), combiner_(combiner), transient_(transientState) {}
    S flatMap(S s) {  // :107-119
        if (!combiner_) return s;
        if (!summary_) summary_ = initial_();
        summary_ = combiner_->reduce(s, *summary_);
        S out = *summary_;
        if (transient_) summary_.reset();
        return out;
    }
    std::vector<S> snapshotState() const {  // :127-130
        return summary_ ? std::vector<S>{*summary_} : std::vector<S>{};
    }
    void restoreState(const std::vector<S>& state) {  // :132-135
        if (!state.empty()) summary_ = state[0];
    }

   private:
    std::function<S()> initial_;
    ReduceFunction<S>* combiner_;
    bool transient_;
    std::optional<S> summary_;
};

template <typename K, typename EV>
class SimpleEdgeStream;

template <typename K, typename EV, typename S, typename T>
class SummaryAggregation {  // …/SummaryAggregation.java:50-91
   public:
    using Emit = std::function<void(const T&)>;
    SummaryAggregation(std::shared_ptr<EdgesFold<K, EV, S>> updateFun, std::shared_ptr<ReduceFunction<S>> combineFun,
                       std::function<T(const S&)> transform, std::function<S()> initialValue, bool transientState)
        : updateFun_(std::move(updateFun)),
          combineFun_(std::move(combineFun)),
          transform_(std::move(transform)),
          initial_(std::move(initialValue)),
          transient_(transientState) {}
    virtual ~SummaryAggregation() = default;
    virtual void run(const SimpleEdgeStream<K, EV>& edgeStream, const Emit& emit) = 0;

    EdgesFold<K, EV, S>* getUpdateFun() const { return updateFun_.get(); }
    ReduceFunction<S>* getCombineFun() const { return combineFun_.get(); }
    bool isTransientState() const { return transient_; }
    // a fresh copy of the initial value: the device summary is created here, on the task side, never in a
    // client-side constructor (the reference Java-serialises its initial value into the job graph)
    S getInitialValue() const { return initial_(); }
    Merger<S> getAggregator() const { return Merger<S>(initial_, combineFun_.get(), transient_); }  // :83-85

   protected:
    T out(const S& s) const {
        if constexpr (std::is_same<S, T>::value) {
            if (!transform_) return s;
        }
        return transform_(s);
    }

   private:
    std::shared_ptr<EdgesFold<K, EV, S>> updateFun_;
    std::shared_ptr<ReduceFunction<S>> combineFun_;
    std::function<T(const S&)> transform_;
    std::function<S()> initial_;
    bool transient_;
};

// SimpleEdgeStream (…/SimpleEdgeStream.java): only the constructors and aggregate() of the hot path.
template <typename K, typename EV>
class SimpleEdgeStream {
   public:
    // EventTime constructor (:86-90): ascending event timestamps in ms, one per edge
    SimpleEdgeStream(std::vector<Edge<K, EV>> edges, std::vector<int64_t> timestamps, int parallelism = 1)
        : edges_(std::move(edges)), ts_(std::move(timestamps)), parallelism_(parallelism < 1 ? 1 : parallelism) {}
    // IngestionTime constructor (:69-73) made deterministic: edge i belongs to window i / edgesPerWindow
    SimpleEdgeStream(std::vector<Edge<K, EV>> edges, uint64_t edgesPerWindow, int parallelism = 1)
        : edges_(std::move(edges)), perWindow_(edgesPerWindow), parallelism_(parallelism < 1 ? 1 : parallelism) {}

    template <typename S, typename T>
    void aggregate(SummaryAggregation<K, EV, S, T>& summaryAggregation,
                   const typename SummaryAggregation<K, EV, S, T>::Emit& emit) const {  // :100-102
        summaryAggregation.run(*this, emit);
    }

    // [begin, end) edge offsets of every non-empty window (tumbling windows of timeMillis)
    std::vector<std::pair<size_t, size_t>> windows(int64_t timeMillis) const {
        std::vector<std::pair<size_t, size_t>> w;
        const size_t n = edges_.size();
        if (n == 0) return w;
        if (!ts_.empty()) {
            size_t b = 0;
            for (size_t i = 1; i <= n; ++i) {
                if (i == n || (ts_[i] - ts_[i] % timeMillis) != (ts_[b] - ts_[b] % timeMillis)) {
                    w.push_back({b, i});
                    b = i;
                }
            }
        } else {
            const uint64_t per = perWindow_ ? perWindow_ : n;
            for (size_t b = 0; b < n; b += per) w.push_back({b, std::min<size_t>(n, b + per)});
        }
        return w;
    }
    const std::vector<Edge<K, EV>>& edges() const { return edges_; }
    int parallelism() const { return parallelism_; }

   private:
    std::vector<Edge<K, EV>> edges_;
    std::vector<int64_t> ts_;
    uint64_t perWindow_ = 0;
    int parallelism_;
};

// SummaryBulkAggregation (…/SummaryBulkAggregation.java:51-131): per window, fold every partition into a fresh
// initial value (keyBy(partition).timeWindow(t).fold), reduce the partials in partition order
// (timeWindowAll(t).reduce), then the Merger; emit once per non-empty window.
template <typename K, typename EV, typename S, typename T>
class SummaryBulkAggregation : public SummaryAggregation<K, EV, S, T> {
   public:
    using Base = SummaryAggregation<K, EV, S, T>;
    SummaryBulkAggregation(std::shared_ptr<EdgesFold<K, EV, S>> updateFun, std::shared_ptr<ReduceFunction<S>> combineFun,
                           std::function<S()> initialVal, int64_t timeMillis, bool transientState,
                           std::function<T(const S&)> transformFun = nullptr)
        : Base(std::move(updateFun), std::move(combineFun), std::move(transformFun), std::move(initialVal),
               transientState),
          timeMillis_(timeMillis) {}

    void run(const SimpleEdgeStream<K, EV>& stream, const typename Base::Emit& emit) override {
        Merger<S> merger = this->getAggregator();
        const int P = stream.parallelism();
        for (auto [b, e] : stream.windows(timeMillis_)) {
            std::optional<S> acc;
            const size_t L = e - b;
            for (int p = 0; p < P; ++p) {
                const size_t pb = b + L * p / P, pe = b + L * (p + 1) / P;
                if (pe == pb) continue;  // a keyed window with no element never fires
                S part = this->getUpdateFun()->foldEdgeBatch(this->getInitialValue(), stream.edges().data() + pb, pe - pb);
                acc = acc ? this->getCombineFun()->reduce(*acc, part) : part;
            }
            emit(this->out(merger.flatMap(*acc)));
        }
    }
    int64_t timeMillis() const { return timeMillis_; }

   protected:
    int64_t timeMillis_;
};

}  // namespace gelly
