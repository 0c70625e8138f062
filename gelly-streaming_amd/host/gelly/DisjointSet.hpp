// gelly/DisjointSet.hpp — C++ host mirror of gelly-streaming's DisjointSet<R>, backed by an MI355X forest.
//
// Reference (`…/` = src/main/java/org/apache/flink/graph/streaming/): …/summaries/DisjointSet.java:30-154.
// Same method names, argument meaning and null/exception behaviour, over the C ABI in include/gelly_cc.h:
//   makeSet (:58-61), find (:71-85, an unseen key -> std::nullopt = Java null), union (:97-123, `union_` here:
//   `union` is a C++ keyword), merge (:132-136), getMatches (:49-51, a lazy read-only view), toString (:139-153).
// Roots are the minimum id of each component (canonical); Java's union-by-rank roots are not part of the
// parity contract. Ids are K values in [0, id_capacity) (u32 on the device).
// Errors from the C ABI throw gelly::GellyException (the Java callbacks are `throws Exception`).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <optional>
#include <sstream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "gelly_cc.h"

namespace gelly {

class GellyException : public std::runtime_error {
   public:
    GellyException(int code, const std::string& what) : std::runtime_error(what), code_(code) {}
    int code() const { return code_; }

   private:
    int code_;
};

inline void check(int rc, const char* fn) {
    if (rc < 0) throw GellyException(rc, std::string(fn) + ": " + gcc_last_error());
}

// one device forest; shared by every DisjointSet handle that refers to the same summary object
struct Forest {
    gcc_forest* h = nullptr;
    uint32_t cap = 0;
    std::vector<uint32_t> labels;  // lazy host view
    bool labels_valid = false;
    Forest(int device, uint32_t id_capacity) : cap(id_capacity) {
        check(gcc_forest_create(device, id_capacity, &h), "gcc_forest_create");
    }
    ~Forest() { gcc_forest_destroy(h); }
    Forest(const Forest&) = delete;
    Forest& operator=(const Forest&) = delete;
    const std::vector<uint32_t>& view() {
        if (!labels_valid) {
            labels.resize(cap);
            check(gcc_forest_labels(h, labels.data(), cap), "gcc_forest_labels");
            labels_valid = true;
        }
        return labels;
    }
};

template <typename K = int64_t>
class DisjointSet {
    static_assert(std::is_integral<K>::value, "DisjointSet ids are integral (u32 on the device)");

   public:
    // `new DisjointSet<>()` (:36-39): the device forest is created here (task side), never in a job graph
    explicit DisjointSet(uint32_t id_capacity, int device = 0) : f_(std::make_shared<Forest>(device, id_capacity)) {}
    // `new DisjointSet<>(Set<R> elements)` (:41-47)
    template <typename It>
    DisjointSet(uint32_t id_capacity, It first, It last, int device = 0) : DisjointSet(id_capacity, device) {
        for (; first != last; ++first) makeSet(*first);
    }

    // read-only Map<K,K> view of getMatches(): key set = ids seen, get(k) = root of k
    class Matches {
       public:
        explicit Matches(std::shared_ptr<Forest> f) : f_(std::move(f)) {}
        uint64_t size() const {
            uint64_t n = 0;
            check(gcc_forest_size(f_->h, &n), "gcc_forest_size");
            return n;
        }
        bool containsKey(K k) const {
            return k >= 0 && (uint64_t)k < f_->cap && f_->view()[(uint32_t)k] != GCC_UNSEEN;
        }
        std::optional<K> get(K k) const {
            if (!containsKey(k)) return std::nullopt;
            return (K)f_->view()[(uint32_t)k];
        }
        std::vector<K> keySet() const {
            std::vector<K> out;
            const auto& lab = f_->view();
            for (uint32_t v = 0; v < f_->cap; ++v)
                if (lab[v] != GCC_UNSEEN) out.push_back((K)v);
            return out;
        }

       private:
        std::shared_ptr<Forest> f_;
    };

    Matches getMatches() const { return Matches(f_); }  // :49-51

    void makeSet(K e) {  // :58-61
        check(gcc_forest_make_set(f_->h, id(e)), "gcc_forest_make_set");
        f_->labels_valid = false;
    }

    std::optional<K> find(K e) const {  // :71-85 (nullopt = Java null for an unseen key)
        if (e < 0 || (uint64_t)e >= f_->cap) return std::nullopt;
        const uint32_t r = f_->view()[(uint32_t)e];
        if (r == GCC_UNSEEN) return std::nullopt;
        return (K)r;
    }

    void union_(K e1, K e2) {  // :97-123
        check(gcc_forest_union(f_->h, id(e1), id(e2)), "gcc_forest_union");
        f_->labels_valid = false;
    }

    void merge(const DisjointSet& other) {  // :132-136
        check(gcc_forest_merge(f_->h, other.f_->h), "gcc_forest_merge");
        f_->labels_valid = false;
    }

    std::string toString() const {  // :139-153 — {root=[members...], ...}, roots = min ids, ascending
        std::map<uint32_t, std::vector<uint32_t>> comps;
        const auto& lab = f_->view();
        for (uint32_t v = 0; v < f_->cap; ++v)
            if (lab[v] != GCC_UNSEEN) comps[lab[v]].push_back(v);
        std::ostringstream os;
        os << "{";
        bool first = true;
        for (const auto& kv : comps) {
            if (!first) os << ", ";
            first = false;
            os << kv.first << "=[";
            for (size_t i = 0; i < kv.second.size(); ++i) os << (i ? ", " : "") << kv.second[i];
            os << "]";
        }
        os << "}";
        return os.str();
    }

    // ---- batch / device extensions of the drop-in ----
    void fold(const uint32_t* pairs, uint64_t n_edges) {  // UpdateCC.foldEdges over a whole host batch
        check(gcc_forest_fold_host(f_->h, pairs, n_edges), "gcc_forest_fold_host");
        f_->labels_valid = false;
    }
    void foldDevice(const uint32_t* d_pairs, uint64_t n_edges) {  // pairs already in HBM
        check(gcc_forest_fold_device(f_->h, d_pairs, n_edges), "gcc_forest_fold_device");
        f_->labels_valid = false;
    }
    const std::vector<uint32_t>& labels() const { return f_->view(); }  // canonical, UNSEEN for unseen ids
    uint64_t numComponents() const {
        uint64_t n = 0;
        check(gcc_forest_count_components(f_->h, &n), "gcc_forest_count_components");
        return n;
    }
    void reset() {  // Merger transientState reset (SummaryAggregation.java:113-115)
        check(gcc_forest_reset(f_->h), "gcc_forest_reset");
        f_->labels_valid = false;
    }
    std::vector<uint32_t> snapshotPairs() const {  // Merger.snapshotState (:127-130): (v, label) of seen v
        std::vector<uint32_t> out;
        const auto& lab = f_->view();
        for (uint32_t v = 0; v < f_->cap; ++v)
            if (lab[v] != GCC_UNSEEN) {
                out.push_back(v);
                out.push_back(lab[v]);
            }
        return out;
    }
    void restorePairs(const std::vector<uint32_t>& pairs) {  // Merger.restoreState (:132-135)
        check(gcc_forest_import_pairs(f_->h, pairs.data(), pairs.size() / 2), "gcc_forest_import_pairs");
        f_->labels_valid = false;
    }
    uint32_t idCapacity() const { return f_->cap; }
    gcc_forest* handle() const { return f_->h; }
    bool sameObject(const DisjointSet& o) const { return f_ == o.f_; }

   private:
    uint32_t id(K e) const {
        if (e < 0 || (uint64_t)e >= f_->cap)
            throw GellyException(GCC_E_INVALID, "vertex id " + std::to_string((long long)e) + " outside [0, " +
                                                    std::to_string(f_->cap) + ")");
        return (uint32_t)e;
    }
    std::shared_ptr<Forest> f_;
};

}  // namespace gelly
