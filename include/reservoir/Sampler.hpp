// reservoir/Sampler.hpp -- C++ host-side mirror of lgbt.princess.reservoir.Sampler over the C ABI
// of libreservoir_hip.so (include/reservoir_hip.h).  Header-only; link with -lreservoir_hip.
//
// Reference: core/src/main/scala/lgbt/princess/reservoir/Sampler.scala (NthPortal/reservoir).
//
//   auto s = reservoir::Sampler<User, int64_t>::apply(100, false, false, [](const User& u) { return u.id; });
//   s->sampleAll(users);                 // Sampler.sampleAll  (Sampler.scala:49-50)
//   std::vector<int64_t> ids = s->result();   // Sampler.result (Sampler.scala:59-60)
//   auto d = reservoir::Sampler<User, int64_t>::distinct(100, false, [](const User& u) { return u.id; });
//
// Names, argument meaning and exceptions follow the reference: IllegalArgumentException for a bad
// maxSampleSize (Sampler.scala:80-81), NullPointerException for a missing map/hash (:82, :94),
// IllegalStateException after result() on a single-use sampler (:186).  `map` runs on the host;
// B (the stored key) must be int32_t (Scala Int) or int64_t (Scala Long).
#pragma once

#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../reservoir_hip.h"

namespace reservoir {

struct IllegalArgumentException : std::invalid_argument {
    using std::invalid_argument::invalid_argument;
};
struct IllegalStateException : std::logic_error {
    using std::logic_error::logic_error;
};
struct NullPointerException : std::invalid_argument {
    using std::invalid_argument::invalid_argument;
};
struct DeviceException : std::runtime_error {
    using std::runtime_error::runtime_error;
};

inline void check(rsv_status st) {
    if (st == RSV_OK) return;
    const std::string msg = rsv_last_error();
    switch (st) {
    case RSV_E_ILLEGAL_ARGUMENT: throw IllegalArgumentException(msg);
    case RSV_E_ILLEGAL_STATE: throw IllegalStateException(msg);
    case RSV_E_NULL_POINTER: throw NullPointerException(msg);
    case RSV_E_OUT_OF_MEMORY: throw std::bad_alloc();
    default: throw DeviceException(std::string(rsv_status_string(st)) + ": " + msg);
    }
}

enum class Engine { PhiloxR = RSV_ENGINE_PHILOX_R, JavaL = RSV_ENGINE_JAVA_L };
enum class Hash {
    Default = RSV_HASH_DEFAULT,    // B#hashCode().toLong (Sampler.scala:75)
    Identity = RSV_HASH_IDENTITY,
    JavaLong = RSV_HASH_JAVA_LONG,
    JavaInt = RSV_HASH_JAVA_INT,
};

// Extensions of the reference factories (all defaulted).
struct Options {
    Engine engine = Engine::PhiloxR;
    bool has_seed = false;
    uint64_t seed = 0;       // default: fresh entropy, like `new Random()` (Sampler.scala:199)
    uint64_t stream_id = 0;  // Philox stream of an Engine::PhiloxR sampler
    int device = -1;         // HIP device ordinal, -1 = current
    // Sampler.distinct tie semantics (rsv_distinct_order): Auto = the reference's sequential heap
    // for colliding hashes (Long#hashCode), order-independent bottom-k for injective ones
    rsv_distinct_order distinct_order = RSV_DISTINCT_AUTO;
};

// trait Sampler[A, B] (Sampler.scala:26-68)
template <class A, class B>
class Sampler {
    static_assert(std::is_same<B, int32_t>::value || std::is_same<B, int64_t>::value,
                  "the GPU engine stores primitive keys: B must be int32_t (Int) or int64_t (Long)");

public:
    using Map = std::function<B(const A&)>;
    using HashFn = std::function<int64_t(const B&)>;

    // Sampler.apply (Sampler.scala:128-136)
    static std::unique_ptr<Sampler> apply(int32_t maxSampleSize, bool preAllocate, bool reusable, Map map,
                                          Options opts = {}) {
        validate(maxSampleSize, map);
        return std::unique_ptr<Sampler>(
            new Sampler(RSV_KIND_ELEMENTS, maxSampleSize, preAllocate, reusable, std::move(map), nullptr,
                        RSV_HASH_DEFAULT, opts));
    }

    // Sampler.distinct (Sampler.scala:171-180) with a recognised hash kind
    static std::unique_ptr<Sampler> distinct(int32_t maxSampleSize, bool reusable, Map map,
                                             Hash hash = Hash::Default, Options opts = {}) {
        validate(maxSampleSize, map);
        return std::unique_ptr<Sampler>(new Sampler(RSV_KIND_DISTINCT, maxSampleSize, false, reusable,
                                                    std::move(map), nullptr, (int32_t)hash, opts));
    }

    // Sampler.distinct with an arbitrary hash function (evaluated on the host, shipped as int64)
    static std::unique_ptr<Sampler> distinct(int32_t maxSampleSize, bool reusable, Map map, HashFn hash,
                                             Options opts = {}) {
        validate(maxSampleSize, map);
        if (!hash) throw NullPointerException("`hash` cannot be `null`");  // Sampler.scala:94
        return std::unique_ptr<Sampler>(new Sampler(RSV_KIND_DISTINCT, maxSampleSize, false, reusable,
                                                    std::move(map), std::move(hash), RSV_HASH_PRECOMPUTED,
                                                    opts));
    }

    ~Sampler() {
        if (h_) rsv_destroy(h_);
    }
    Sampler(const Sampler&) = delete;
    Sampler& operator=(const Sampler&) = delete;

    // Sampler.sample (Sampler.scala:37-38)
    void sample(const A& element) {
        const B key = map_(element);
        if (hash_) {
            const int64_t hv = hash_(key);
            check(rsv_sample(h_, &key, &hv));
        } else {
            check(rsv_sample(h_, &key, nullptr));
        }
    }

    // Sampler.sampleAll (Sampler.scala:49-50): one batch through the ABI
    template <class Range>
    void sampleAll(const Range& elements) {
        if (!isOpen()) throw IllegalStateException("use of sampler after calling `result()`");
        keys_.clear();
        hashes_.clear();
        for (const auto& e : elements) {
            keys_.push_back(map_(e));
            if (hash_) hashes_.push_back(hash_(keys_.back()));
        }
        check(rsv_sample_batch(h_, keys_.data(), (int64_t)keys_.size(), RSV_MEM_HOST,
                               hash_ ? hashes_.data() : nullptr));
    }

    // keys already extracted and resident in HBM (device pointer): sampled in place
    void sampleAllDevice(const B* keys_dev, int64_t n) {
        check(rsv_sample_batch(h_, keys_dev, n, RSV_MEM_DEVICE, nullptr));
    }

    // Sampler.result (Sampler.scala:59-60)
    std::vector<B> result() {
        std::vector<B> out((size_t)k_);
        int64_t n = 0;
        check(rsv_result(h_, out.data(), k_, &n));
        out.resize((size_t)n);
        return out;
    }

    // Sampler.isOpen (Sampler.scala:67)
    bool isOpen() const { return rsv_is_open(h_) != 0; }

    int64_t count() const { return rsv_count(h_); }
    rsv_sampler* handle() const { return h_; }

private:
    static void validate(int32_t k, const Map& map) {  // validateSharedParams (Sampler.scala:79-83)
        if (k > 2147483647 - 2) throw IllegalArgumentException("requirement failed: maxSampleSize exceeds VM limit");
        if (k <= 0) throw IllegalArgumentException("requirement failed: maxSampleSize must be positive");
        if (!map) throw NullPointerException("`map` cannot be `null`");
    }

    Sampler(int32_t kind, int32_t k, bool preAllocate, bool reusable, Map map, HashFn hash, int32_t hash_kind,
            const Options& opts)
        : k_(k), map_(std::move(map)), hash_(std::move(hash)) {
        rsv_config cfg;
        check(rsv_config_init(&cfg));
        cfg.kind = kind;
        cfg.max_sample_size = k;
        cfg.key_width = (int32_t)sizeof(B);
        cfg.reusable = reusable ? 1 : 0;
        cfg.pre_allocate = preAllocate ? 1 : 0;
        cfg.engine = (int32_t)opts.engine;
        cfg.hash_kind = hash_kind;
        cfg.device = opts.device;
        cfg.distinct_order = (int32_t)opts.distinct_order;
        if (opts.has_seed) {
            cfg.seed = opts.seed;
        } else {
            std::random_device rd;
            cfg.seed = ((uint64_t)rd() << 32) ^ rd();
        }
        cfg.stream_id = opts.stream_id;
        check(rsv_create(&cfg, &h_));
    }

    rsv_sampler* h_ = nullptr;
    int32_t k_;
    Map map_;
    HashFn hash_;
    std::vector<B> keys_;
    std::vector<int64_t> hashes_;
};

}  // namespace reservoir
