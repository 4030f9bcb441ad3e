// test_ffm_sequence.cpp -- replays, on the GPU and without a JDK, exactly the call sequences the two
// JVM bindings drive:
//   ffm   FfmMirror below: statement for statement the Panama FFM binding
//         bindings/scala/ffm/lgbt/princess/reservoir/gpu/ffm/FfmSampler.scala over the raw C ABI
//         (stage_acquire / commit per ~1 Mi keys, open tracked on the JVM side, the single-use
//         result() destroys the handle and nothing touches it afterwards)
//   jni   bindings/jvm/rsv_jvm.c, the session logic every JNI native method of
//         bindings/jni/reservoir_jni.c consists of (sample per element, sampleAll over arrays)
//   abi   per-element rsv_sample (the engine's own staging), for the akka path at C5's k = 1 Mi
//   fidx  FfmSampler.sampleAll over an IndexedSeq (rsv_sample_indexed + rsv_fill_slots): a few
//         elements per element first, then the rest of the sequence by index -- map (here: the
//         key of offset i) runs only for the slots' new holders, no key buffer for the sequence
//   jidx  the same through rsv_jvm (JniSampler.sampleAll's natives)
//   fobj  ObjectSampler.scala (a Sampler[A, B] for any B: the B values stay on the JVM) over the
//         FFM downcalls: buffered sample() batches and IndexedSeq batches by index only
//         (rsv_sample_indexed + rsv_commit_indexed), a throwing map undone by rsv_abort_indexed
//   jobj  the same through rsv_jvm (JniIndexOps)
// Each case line of argv[1] names the sampler, its keys (splitmix64(base + i), or a binary key file)
// and a binary file with the oracle's expected result (tests/test_gpu_ffm.py writes them);
// distinct results compare as sets.
// Prints PASS/FAIL per case; exit status = number of failures.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../bindings/jvm/rsv_jvm.h"
#include "../../include/reservoir_hip.h"

static int failures = 0;
#define EXPECT(c, what)                                                                  \
    do {                                                                                 \
        if (!(c)) {                                                                      \
            std::printf("FAIL %s: %s (%s:%d)\n", what, #c, __FILE__, __LINE__);          \
            ++failures;                                                                  \
        }                                                                                \
    } while (0)

struct JvmException : std::runtime_error {
    rsv_status status;
    JvmException(rsv_status st, const std::string& m) : std::runtime_error(m), status(st) {}
};

// Native.check of FfmSampler.scala: status -> the reference's exception
static void check(rsv_status st) {
    if (st != RSV_OK) throw JvmException(st, rsv_last_error());
}

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// ---- FfmMirror: FfmSampler.scala, line for line ------------------------------------------------
struct FfmMirror {
    rsv_sampler* handle = nullptr;
    bool open = true;  // tracked on the JVM side: isOpen makes no downcall
    bool reusable, precomputed;
    int width, k;
    uint8_t* stage = nullptr;
    int64_t* stage_hash = nullptr;
    int64_t cap = 0, filled = 0;

    FfmMirror(const rsv_config& c)
        : reusable(c.reusable != 0), precomputed(c.kind == RSV_KIND_DISTINCT && c.hash_kind == RSV_HASH_PRECOMPUTED),
          width(c.key_width), k(c.max_sample_size) {
        check(rsv_create(&c, &handle));
    }
    void next_stage() {
        if (filled > 0) {
            const int64_t f = filled;
            filled = 0;
            cap = 0;
            check(rsv_stage_commit(handle, f));
        }
        void* keys = nullptr;
        int64_t* hashes = nullptr;
        check(rsv_stage_acquire(handle, &keys, precomputed ? &hashes : nullptr, &cap));
        stage = (uint8_t*)keys;
        stage_hash = hashes;
    }
    void sample(const void* key, int64_t hash) {
        if (!open) throw JvmException(RSV_E_ILLEGAL_STATE, "use of sampler after calling `result()`");
        if (filled == cap) next_stage();
        std::memcpy(stage + filled * width, key, (size_t)width);
        if (precomputed) stage_hash[filled] = hash;
        filled += 1;
    }
    // sampleAll over an IndexedSeq of n elements; key_at(i, dst) is `map(seq(i))`.  Returns the
    // number of elements mapped.
    template <class KeyAt>
    int64_t sample_all_indexed(int64_t n, KeyAt key_at) {
        if (!open) throw JvmException(RSV_E_ILLEGAL_STATE, "use of sampler after calling `result()`");
        if (filled > 0) {  // the staged keys come first in index order
            const int64_t f = filled;
            filled = 0;
            check(rsv_stage_commit(handle, f));
        }
        cap = 0;
        std::vector<int64_t> offsets((size_t)k);
        check(rsv_sample_indexed(handle, n, offsets.data()));
        std::vector<uint8_t> ks((size_t)k * width);
        int64_t mapped = 0;
        try {
            for (int j = 0; j < k; ++j) {
                const int64_t o = offsets[(size_t)j];
                if (o >= 0) {
                    key_at(o, ks.data() + (size_t)j * width);
                    ++mapped;
                }
            }
        } catch (...) {  // `map` threw: drop the batch, keep the sampler usable, propagate
            check(rsv_abort_indexed(handle));
            throw;
        }
        check(rsv_fill_slots(handle, ks.data()));
        return mapped;
    }
    std::vector<uint8_t> result(int64_t* n_out) {
        if (!open) throw JvmException(RSV_E_ILLEGAL_STATE, "use of sampler after calling `result()`");
        if (filled > 0) {
            const int64_t f = filled;
            filled = 0;
            check(rsv_stage_commit(handle, f));
        }
        cap = 0;  // the staging pointers die with the next call on the handle
        std::vector<uint8_t> out((size_t)k * width);
        int64_t n = 0;
        check(rsv_result(handle, out.data(), k, &n));
        out.resize((size_t)n * width);
        if (!reusable) {  // SingleUse.close: the handle is destroyed and never touched again
            open = false;
            rsv_destroy(handle);
            handle = nullptr;
        }
        *n_out = n;
        return out;
    }
    ~FfmMirror() {
        if (handle) rsv_destroy(handle);  // the Cleaner of a reusable sampler
    }
};

// ---- ObjectMirror: ObjectSampler.scala (a Sampler[A, B] for any B), line for line ----------------
// The B values are int64 "references" here; the IndexOps are the FFM downcalls (FfmIndexOps) or the
// rsv_jvm session functions every JNI native of JniIndexOps calls.
struct MapThrew : std::runtime_error {
    MapThrew() : std::runtime_error("map threw") {}
};

struct ObjectMirror {
    static constexpr int Batch = 65536;
    bool via_jvm, reusable, open = true, aliased = false;
    int k;
    rsv_sampler* handle = nullptr;  // FfmIndexOps
    rsv_jvm js;                     // JniIndexOps
    std::vector<int64_t> slots, pending, offsets;
    int n = 0;
    int64_t count = 0;

    ObjectMirror(const rsv_config& c, bool jvm) : via_jvm(jvm), reusable(c.reusable != 0), k(c.max_sample_size) {
        rsv_config cfg = c;
        cfg.key_width = 8;  // never used for keys
        if (via_jvm) check(rsv_jvm_create(&js, &cfg));
        else check(rsv_create(&cfg, &handle));
        slots.resize((size_t)std::min(16, k));
        pending.resize(Batch);
    }
    ~ObjectMirror() { release(); }
    void release() {
        if (via_jvm) rsv_jvm_destroy(&js);
        else if (handle) rsv_destroy(handle);
        handle = nullptr;
    }
    // IndexOps
    void sample_indexed(int64_t len, int64_t* o) {
        check(via_jvm ? rsv_jvm_sample_indexed(&js, len, o) : rsv_sample_indexed(handle, len, o));
    }
    void commit() { check(via_jvm ? rsv_jvm_commit_indexed(&js) : rsv_commit_indexed(handle)); }
    void abort() { check(via_jvm ? rsv_jvm_abort_indexed(&js) : rsv_abort_indexed(handle)); }

    void ensure_size(int j) {
        if ((int)slots.size() <= j) {
            const size_t len = slots.size();
            const size_t grow = std::min<size_t>((size_t)k, len << 1);
            slots.resize(std::max<size_t>(grow, (size_t)j + 1));
        }
    }
    int64_t* offset_array() {
        if (offsets.empty()) offsets.resize((size_t)k);
        return offsets.data();
    }
    void flush() {
        if (n == 0) return;
        int64_t* o = offset_array();
        sample_indexed(n, o);
        commit();
        aliased = false;  // (a copy in the JVM; the vector here is never shared)
        for (int j = 0; j < k; ++j)
            if (o[j] >= 0) {
                ensure_size(j);
                slots[(size_t)j] = pending[(size_t)o[j]];
            }
        count += n;
        n = 0;
    }
    void sample(int64_t b) {
        if (!open) throw JvmException(RSV_E_ILLEGAL_STATE, "use of sampler after calling `result()`");
        pending[(size_t)n++] = b;
        if (n == Batch) flush();
    }
    // sampleAll over a known-size IndexedSeq; map(i) = the element at offset i (may throw MapThrew).
    // Returns the number of map calls.
    template <class Map>
    int64_t sample_all_indexed(int64_t len, Map map) {
        if (!open) throw JvmException(RSV_E_ILLEGAL_STATE, "use of sampler after calling `result()`");
        flush();
        int64_t* o = offset_array();
        sample_indexed(len, o);
        std::vector<int> js_;
        std::vector<int64_t> vals;
        int64_t calls = 0;
        try {
            for (int j = 0; j < k; ++j)
                if (o[j] >= 0) {
                    ++calls;
                    vals.push_back(map(o[j]));
                    js_.push_back(j);
                }
        } catch (...) {
            abort();
            throw;
        }
        commit();
        for (size_t c = 0; c < js_.size(); ++c) {
            ensure_size(js_[c]);
            slots[(size_t)js_[c]] = vals[c];
        }
        count += len;
        return calls;
    }
    std::vector<int64_t> result() {
        if (!open) throw JvmException(RSV_E_ILLEGAL_STATE, "use of sampler after calling `result()`");
        flush();
        const int64_t m = std::min<int64_t>(count, k);
        std::vector<int64_t> out(slots.begin(), slots.begin() + m);
        if (!reusable) {
            open = false;
            release();
        }
        return out;
    }
};

// ---- cases ---------------------------------------------------------------------------------------
struct Case {
    std::string name, path, expected, keyfile;  // keyfile (optional): the keys, else splitmix64(base + i)
    std::vector<uint8_t> keys;
    int kind, k, kw, reusable, hash_kind, order, engine;
    uint64_t seed, stream, base;
    int64_t n;
};

static std::vector<uint8_t> read_file(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

// key i of the case, written into `dst` (kw bytes), and its precomputed hash (31 x + 7)
static int64_t make_key(const Case& c, int64_t i, void* dst) {
    if (!c.keys.empty()) {
        std::memcpy(dst, c.keys.data() + i * c.kw, (size_t)c.kw);
        int64_t v = 0;
        if (c.kw >= 8) std::memcpy(&v, dst, 8);  // byte keys: the hash reads the first word
        else {
            int32_t w;
            std::memcpy(&w, dst, 4);
            v = w;
        }
        return (int64_t)((uint64_t)v * 31u + 7u);
    }
    const int64_t v = (int64_t)splitmix64(c.base + (uint64_t)i);
    if (c.kw > 8) {  // byte keys (UUID): [v, ~v], then zero words
        std::memset(dst, 0, (size_t)c.kw);
        const uint64_t w[2] = {(uint64_t)v, ~(uint64_t)v};
        std::memcpy(dst, w, 16);
        return (int64_t)((uint64_t)v * 31u + 7u);
    }
    if (c.kw == 8) {
        std::memcpy(dst, &v, 8);
        return (int64_t)((uint64_t)v * 31u + 7u);
    }
    const int32_t w = (int32_t)(v >> 33);
    std::memcpy(dst, &w, 4);
    return (int64_t)((uint64_t)(int64_t)w * 31u + 7u);
}

static bool same(const Case& c, std::vector<uint8_t> got, int64_t n) {
    std::vector<uint8_t> want = read_file(c.expected);
    if ((int64_t)want.size() != n * c.kw || got.size() != want.size()) {
        std::printf("  %s: size %lld keys, expected %zu\n", c.name.c_str(), (long long)n, want.size() / c.kw);
        return false;
    }
    if (c.kind == RSV_KIND_DISTINCT) {  // HashSet order in the reference: compare as sets
        auto sort_keys = [&](std::vector<uint8_t>& b) {
            if (c.kw == 8) std::sort((int64_t*)b.data(), (int64_t*)b.data() + n);
            else if (c.kw == 4) std::sort((int32_t*)b.data(), (int32_t*)b.data() + n);
            else {  // byte keys: sort the rows as strings
                std::vector<std::string> rows((size_t)n);
                for (int64_t i = 0; i < n; ++i) rows[(size_t)i].assign((const char*)b.data() + i * c.kw, (size_t)c.kw);
                std::sort(rows.begin(), rows.end());
                for (int64_t i = 0; i < n; ++i) std::memcpy(b.data() + i * c.kw, rows[(size_t)i].data(), (size_t)c.kw);
            }
        };
        sort_keys(got);
        sort_keys(want);
    }
    return got == want;
}

static rsv_config config_of(const Case& c) {
    rsv_config cfg;
    rsv_config_init(&cfg);
    cfg.kind = c.kind;
    cfg.max_sample_size = c.k;
    cfg.key_width = c.kw;
    cfg.reusable = c.reusable;
    cfg.hash_kind = c.hash_kind;
    cfg.distinct_order = c.order;
    cfg.engine = c.engine;
    cfg.seed = c.seed;
    cfg.stream_id = c.stream;
    return cfg;
}

static void run_ffm(const Case& c) {
    FfmMirror s(config_of(c));
    uint8_t key[256];
    for (int64_t i = 0; i < c.n; ++i) {
        const int64_t h = make_key(c, i, key);
        s.sample(key, h);
    }
    int64_t n = 0;
    std::vector<uint8_t> r = s.result(&n);
    EXPECT(same(c, r, n), c.name.c_str());
    if (!c.reusable) {
        EXPECT(!s.open && s.handle == nullptr, c.name.c_str());  // isOpen == false, handle gone
        bool ise = false;
        try {
            s.sample(key, 0);
        } catch (const JvmException& e) {
            ise = e.status == RSV_E_ILLEGAL_STATE;
        }
        EXPECT(ise, c.name.c_str());
        ise = false;
        try {
            s.result(&n);
        } catch (const JvmException& e) {
            ise = e.status == RSV_E_ILLEGAL_STATE;
        }
        EXPECT(ise, c.name.c_str());
    } else {  // MultiResult: still open, the next result equals the last, sampling continues
        int64_t n2 = 0;
        std::vector<uint8_t> r2 = s.result(&n2);
        EXPECT(s.open && n2 == n && r2 == r, c.name.c_str());
        s.sample(key, 0);
        s.result(&n2);
        EXPECT(s.open, c.name.c_str());
    }
}

static void run_jni(const Case& c) {
    rsv_jvm s;
    const rsv_config cfg = config_of(c);
    rsv_status st = rsv_jvm_create(&s, &cfg);
    EXPECT(st == RSV_OK, c.name.c_str());
    if (st != RSV_OK) return;
    // sampleAll over JVM arrays of 65536 keys (JniSampler's buffer), the odd tail per element
    const int64_t B = 65536;
    std::vector<uint8_t> buf((size_t)B * c.kw);
    std::vector<int64_t> hb((size_t)B);
    int64_t i = 0;
    for (; i + B <= c.n; i += B) {
        for (int64_t t = 0; t < B; ++t) hb[(size_t)t] = make_key(c, i + t, buf.data() + t * c.kw);
        st = rsv_jvm_sample_array(&s, buf.data(), s.precomputed ? hb.data() : nullptr, B);
        EXPECT(st == RSV_OK, c.name.c_str());
    }
    uint8_t key[256];
    for (; i < c.n; ++i) {
        const int64_t h = make_key(c, i, key);
        st = rsv_jvm_sample(&s, key, h);
        EXPECT(st == RSV_OK, c.name.c_str());
    }
    std::vector<uint8_t> out((size_t)c.k * c.kw);
    int64_t n = 0;
    st = rsv_jvm_result(&s, out.data(), c.k, &n);
    EXPECT(st == RSV_OK, c.name.c_str());
    out.resize((size_t)n * c.kw);
    EXPECT(same(c, out, n), c.name.c_str());
    if (!c.reusable) {
        EXPECT(rsv_jvm_is_open(&s) == 0 && s.h == nullptr, c.name.c_str());
        st = rsv_jvm_sample(&s, key, 0);
        EXPECT(st == RSV_E_ILLEGAL_STATE, c.name.c_str());
        EXPECT(std::strstr(rsv_jvm_last_error(), "result()") != nullptr, c.name.c_str());
        EXPECT(std::strcmp(rsv_jvm_exception_class(st), "java/lang/IllegalStateException") == 0, c.name.c_str());
        st = rsv_jvm_result(&s, out.data(), c.k, &n);
        EXPECT(st == RSV_E_ILLEGAL_STATE, c.name.c_str());
        void* p = nullptr;
        int64_t cap = 0;
        EXPECT(rsv_jvm_stage_acquire(&s, &p, &cap) == RSV_E_ILLEGAL_STATE, c.name.c_str());
    } else {
        EXPECT(rsv_jvm_is_open(&s) == 1, c.name.c_str());
        std::vector<uint8_t> out2((size_t)c.k * c.kw);
        int64_t n2 = 0;
        EXPECT(rsv_jvm_result(&s, out2.data(), c.k, &n2) == RSV_OK, c.name.c_str());
        out2.resize((size_t)n2 * c.kw);
        EXPECT(n2 == n && out2 == out, c.name.c_str());
    }
    rsv_jvm_destroy(&s);
}

static void run_abi(const Case& c) {  // per-element rsv_sample: the engine stages and flushes
    const rsv_config cfg = config_of(c);
    rsv_sampler* h = nullptr;
    check(rsv_create(&cfg, &h));
    uint8_t key[256];
    for (int64_t i = 0; i < c.n; ++i) {
        int64_t hv = make_key(c, i, key);
        rsv_status st = rsv_sample(h, key, &hv);
        if (st != RSV_OK) {
            EXPECT(st == RSV_OK, c.name.c_str());
            break;
        }
    }
    std::vector<uint8_t> out((size_t)c.k * c.kw);
    int64_t n = 0;
    EXPECT(rsv_result(h, out.data(), c.k, &n) == RSV_OK, c.name.c_str());
    out.resize((size_t)n * c.kw);
    EXPECT(same(c, out, n), c.name.c_str());
    EXPECT(rsv_is_open(h) == c.reusable, c.name.c_str());
    rsv_destroy(h);
}

// sampleAll over an IndexedSeq: the first `pre` elements per element, the rest by index.  The
// sequence is virtual (key i = make_key(c, i)): no key buffer exists for it.
static void run_indexed(const Case& c, bool ffm) {
    const int64_t pre = std::min<int64_t>(c.n, 5);
    uint8_t key[256];
    int64_t mapped = 0;
    std::vector<uint8_t> out;
    int64_t n = 0;
    if (ffm) {
        FfmMirror s(config_of(c));
        for (int64_t i = 0; i < pre; ++i) {
            const int64_t h = make_key(c, i, key);
            s.sample(key, h);
        }
        mapped = s.sample_all_indexed(c.n - pre, [&](int64_t o, uint8_t* dst) { make_key(c, pre + o, dst); });
        out = s.result(&n);
    } else {
        rsv_jvm s;
        const rsv_config cfg = config_of(c);
        rsv_status st = rsv_jvm_create(&s, &cfg);
        EXPECT(st == RSV_OK, c.name.c_str());
        if (st != RSV_OK) return;
        for (int64_t i = 0; i < pre; ++i) {
            const int64_t h = make_key(c, i, key);
            EXPECT(rsv_jvm_sample(&s, key, h) == RSV_OK, c.name.c_str());
        }
        std::vector<int64_t> offsets((size_t)c.k);
        EXPECT(rsv_jvm_sample_indexed(&s, c.n - pre, offsets.data()) == RSV_OK, c.name.c_str());
        // a call before the owed keys arrive is an IllegalStateException; the sampler is unharmed
        std::vector<uint8_t> probe((size_t)c.k * c.kw);
        int64_t pn = 0;
        EXPECT(rsv_jvm_result(&s, probe.data(), c.k, &pn) == RSV_E_ILLEGAL_STATE, c.name.c_str());
        std::vector<uint8_t> ks((size_t)c.k * c.kw);
        for (int j = 0; j < c.k; ++j)
            if (offsets[(size_t)j] >= 0) {
                make_key(c, pre + offsets[(size_t)j], ks.data() + (size_t)j * c.kw);
                ++mapped;
            }
        EXPECT(rsv_jvm_fill_slots(&s, ks.data()) == RSV_OK, c.name.c_str());
        EXPECT(rsv_jvm_fill_slots(&s, ks.data()) == RSV_E_ILLEGAL_STATE, c.name.c_str());  // nothing owed now
        out.resize((size_t)c.k * c.kw);
        EXPECT(rsv_jvm_result(&s, out.data(), c.k, &n) == RSV_OK, c.name.c_str());
        out.resize((size_t)n * c.kw);
        rsv_jvm_destroy(&s);
    }
    EXPECT(same(c, out, n), c.name.c_str());
    EXPECT(mapped <= c.k, c.name.c_str());  // map ran only for the reservoir's new holders
    std::printf("  %s: %lld of %lld indexed elements mapped\n", c.name.c_str(), (long long)mapped,
                (long long)(c.n - pre));
}

// A Sampler[A, B] for any B (ObjectSampler): element i of the stream is the "reference" i, so the
// reservoir must hold the oracle's last-writer indices.  The first `pre` elements go through
// sample() (one full 65536-element buffer flushed by index, the rest buffered), then the remaining
// ones as an IndexedSeq whose map throws on its third call (the batch is dropped, the exception
// propagates), then the same IndexedSeq again with a map that succeeds.
static void run_objects(const Case& c, bool jvm) {
    ObjectMirror s(config_of(c), jvm);
    const int64_t pre = std::min<int64_t>(c.n, 100003);
    for (int64_t i = 0; i < pre; ++i) s.sample(i);
    const int64_t rest = c.n - pre;
    int64_t calls = 0;
    if (rest > 0) {
        int64_t seen = 0;
        bool threw = false;
        try {
            s.sample_all_indexed(rest, [&](int64_t o) -> int64_t {
                if (++seen == 3) throw MapThrew();
                return pre + o;
            });
        } catch (const MapThrew&) {
            threw = true;
        }
        EXPECT(threw || seen < 3, c.name.c_str());
        if (!jvm && pre > 0) {  // the handle's slots hold no keys now: keyed calls are refused
            int64_t x = 0, nn = 0;
            EXPECT(rsv_sample(s.handle, &x, nullptr) == RSV_E_ILLEGAL_STATE, c.name.c_str());
            EXPECT(rsv_sample_batch(s.handle, &x, 1, RSV_MEM_HOST, nullptr) == RSV_E_ILLEGAL_STATE, c.name.c_str());
            EXPECT(rsv_result(s.handle, &x, 1, &nn) == RSV_E_ILLEGAL_STATE, c.name.c_str());
            EXPECT(rsv_commit_indexed(s.handle) == RSV_E_ILLEGAL_STATE, c.name.c_str());  // nothing pending
        }
        calls = s.sample_all_indexed(rest, [&](int64_t o) -> int64_t { return pre + o; });
    }
    std::vector<int64_t> got = s.result();
    const std::vector<uint8_t> wb = read_file(c.expected);
    std::vector<int64_t> want(wb.size() / 8);
    std::memcpy(want.data(), wb.data(), wb.size());
    EXPECT(got == want, c.name.c_str());
    EXPECT(calls <= c.k, c.name.c_str());  // map ran only for the reservoir's new holders
    if (c.reusable) {
        EXPECT(s.result() == got && s.open, c.name.c_str());
    } else {
        bool ise = false;
        try {
            s.sample(0);
        } catch (const JvmException& e) {
            ise = e.status == RSV_E_ILLEGAL_STATE;
        }
        EXPECT(ise && !s.open, c.name.c_str());
    }
    std::printf("  %s: %lld indexed elements, map called %lld times\n", c.name.c_str(), (long long)rest,
                (long long)calls);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s cases.txt\n", argv[0]);
        return 2;
    }
    // the exception mapping of both bindings (Sampler.scala:80-81)
    for (int bad : {0, -1, 2147483647}) {
        rsv_config cfg;
        rsv_config_init(&cfg);
        cfg.max_sample_size = bad;
        rsv_jvm s;
        const rsv_status st = rsv_jvm_create(&s, &cfg);
        EXPECT(st == RSV_E_ILLEGAL_ARGUMENT, "create with a bad maxSampleSize");
        EXPECT(std::strcmp(rsv_jvm_exception_class(st), "java/lang/IllegalArgumentException") == 0, "IAE class");
    }
    std::ifstream f(argv[1]);
    std::string line;
    while (std::getline(f, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::istringstream is(line);
        Case c;
        is >> c.name >> c.path >> c.kind >> c.k >> c.kw >> c.reusable >> c.hash_kind >> c.order >> c.engine >> c.seed >>
            c.stream >> c.n >> c.base >> c.expected;
        if (is >> c.keyfile) c.keys = read_file(c.keyfile);
        const int before = failures;
        try {
            if (c.path == "ffm") run_ffm(c);
            else if (c.path == "jni") run_jni(c);
            else if (c.path == "abi") run_abi(c);
            else if (c.path == "fidx") run_indexed(c, true);
            else if (c.path == "jidx") run_indexed(c, false);
            else if (c.path == "fobj") run_objects(c, false);
            else if (c.path == "jobj") run_objects(c, true);
            else throw std::runtime_error("unknown path " + c.path);
        } catch (const std::exception& e) {
            std::printf("FAIL %s: exception %s\n", c.name.c_str(), e.what());
            ++failures;
        }
        if (failures == before) std::printf("PASS %s\n", c.name.c_str());
        std::fflush(stdout);
    }
    return failures;
}
