// bench_c5.cpp -- config C5: a per-element source feeding the sampler through
// the C ABI one element at a time (what the akka operator's onPush does, SampleImpl.scala:27-31),
// k = 1M.  Measures the sustained element rate of rsv_sample (pinned double-buffered staging,
// asynchronous flushes) and the end-to-end time including result().
// Build: g++ -O3 -std=c++17 -I include tools/bench_c5.cpp -L reservoir_amd -lreservoir_hip \
//            -Wl,-rpath,'$ORIGIN/../reservoir_amd' -o tools/bench_c5   (__graft_entry__.build does this)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "reservoir/Sampler.hpp"

static uint64_t splitmix(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 200000000LL;
    const int32_t k = argc > 2 ? atoi(argv[2]) : 1 << 20;
    std::vector<int64_t> src(1 << 24);
    for (size_t i = 0; i < src.size(); ++i) src[i] = (int64_t)splitmix(0x5EED0000ULL + i);
    for (int engine = 0; engine < 2; ++engine) {
        rsv_config cfg;
        reservoir::check(rsv_config_init(&cfg));
        cfg.max_sample_size = k;
        cfg.engine = engine;
        cfg.seed = 7;
        rsv_sampler* s = nullptr;
        reservoir::check(rsv_create(&cfg, &s));
        const size_t mask = src.size() - 1;
        // warm-up: first 2 batches
        for (int64_t i = 0; i < (2 << 20); ++i) reservoir::check(rsv_sample(s, &src[i & mask], nullptr));
        auto t0 = std::chrono::steady_clock::now();
        for (int64_t i = 0; i < n; ++i) reservoir::check(rsv_sample(s, &src[i & mask], nullptr));
        auto t1 = std::chrono::steady_clock::now();
        std::vector<int64_t> out((size_t)k);
        int64_t m = 0;
        reservoir::check(rsv_result(s, out.data(), k, &m));
        auto t2 = std::chrono::steady_clock::now();
        const double ds = std::chrono::duration<double>(t1 - t0).count();
        const double de = std::chrono::duration<double>(t2 - t0).count();
        std::printf("{\"config\": \"C5 per-element rsv_sample, k=%d, engine=%s\", \"elements\": %lld, "
                    "\"sustained_Melem_s\": %.1f, \"end_to_end_Melem_s\": %.1f, \"result_n\": %lld}\n",
                    k, engine ? "java_l" : "philox_r", (long long)n, n / ds / 1e6, n / de / 1e6, (long long)m);
        rsv_destroy(s);
    }
    // zero-copy pinned batches: the source writes each key straight into the staging buffer
    // (rsv_stage_acquire / rsv_stage_commit), one ABI call per ~1 Mi keys instead of per key
    for (int engine = 0; engine < 2; ++engine) {
        rsv_config cfg;
        reservoir::check(rsv_config_init(&cfg));
        cfg.max_sample_size = k;
        cfg.engine = engine;
        cfg.seed = 7;
        rsv_sampler* s = nullptr;
        reservoir::check(rsv_create(&cfg, &s));
        const size_t mask = src.size() - 1;
        auto feed = [&](int64_t count) {
            int64_t i = 0;
            while (i < count) {
                void* buf = nullptr;
                int64_t cap = 0;
                reservoir::check(rsv_stage_acquire(s, &buf, nullptr, &cap));
                const int64_t c = std::min<int64_t>(cap, count - i);
                int64_t* kb = (int64_t*)buf;
                for (int64_t t = 0; t < c; ++t) kb[t] = src[(size_t)(i + t) & mask];  // the "map" of each element
                reservoir::check(rsv_stage_commit(s, c));
                i += c;
            }
        };
        feed(2 << 20);
        auto t0 = std::chrono::steady_clock::now();
        feed(n);
        auto t1 = std::chrono::steady_clock::now();
        std::vector<int64_t> out((size_t)k);
        int64_t m = 0;
        reservoir::check(rsv_result(s, out.data(), k, &m));
        auto t2 = std::chrono::steady_clock::now();
        const double ds = std::chrono::duration<double>(t1 - t0).count();
        const double de = std::chrono::duration<double>(t2 - t0).count();
        std::printf("{\"config\": \"C5 zero-copy pinned batches (rsv_stage_acquire/commit), k=%d, engine=%s\", "
                    "\"elements\": %lld, \"sustained_Melem_s\": %.1f, \"end_to_end_Melem_s\": %.1f, "
                    "\"result_n\": %lld}\n",
                    k, engine ? "java_l" : "philox_r", (long long)n, n / ds / 1e6, n / de / 1e6, (long long)m);
        rsv_destroy(s);
    }
    // the source alone: the same loop writing the same pinned staging memory with no sampler work
    // (nothing committed) -- the host-side ceiling of the zero-copy legs above
    {
        rsv_config cfg;
        reservoir::check(rsv_config_init(&cfg));
        cfg.max_sample_size = k;
        rsv_sampler* s = nullptr;
        reservoir::check(rsv_create(&cfg, &s));
        void* buf = nullptr;
        int64_t cap = 0;
        reservoir::check(rsv_stage_acquire(s, &buf, nullptr, &cap));
        int64_t* kb = (int64_t*)buf;
        const size_t mask = src.size() - 1;
        auto t0 = std::chrono::steady_clock::now();
        for (int64_t i = 0; i < n;) {
            const int64_t c = std::min<int64_t>(cap, n - i);
            for (int64_t t = 0; t < c; ++t) kb[t] = src[(size_t)(i + t) & mask];
            asm volatile("" ::: "memory");  // every chunk's stores happen
            i += c;
        }
        auto t1 = std::chrono::steady_clock::now();
        volatile int64_t sink = kb[cap - 1];
        (void)sink;
        const double ds = std::chrono::duration<double>(t1 - t0).count();
        std::printf("{\"config\": \"C5 source alone: the zero-copy legs' fill loop into the same pinned staging buffer, "
                    "no sampler work\", \"elements\": %lld, \"sustained_Melem_s\": %.1f}\n",
                    (long long)n, n / ds / 1e6);
        rsv_destroy(s);
    }
    return 0;
}
