// micro_heap_wide.cpp -- development probe (not part of the library): the byte-key replica's
// heap-only replay (HostValuesWide, rsv_host_values.h) over a synthetic first-occurrence log shaped
// like the C4 UUID hash-twin share (1.36 M rows of 16 B, k = 65536, hashes falling with arrival like
// the scheduled pass's bounds).  sample_first (a pool slot + row copy per replacement) vs
// sample_first_at + adopt (log positions during the run); both heaps must be identical (checked).
//   g++ -O3 -march=native -std=c++17 tools/micro_heap_wide.cpp -o /tmp/micro_heap_wide
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../reservoir_amd/csrc/rsv_host_values.h"

static uint64_t smix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const int64_t k = 65536, W = 2, N = argc > 1 ? atoll(argv[1]) : 1360000;
    std::vector<int64_t> h((size_t)N);
    std::vector<uint64_t> rows((size_t)(N * W));
    const double span = 18446744073709551616.0;
    for (int64_t t = 0; t < N; ++t) {
        // the bound the row passed: ~2k of the range early, falling like 1 / arrival later
        const double frac = std::min(1.0, 2.0 * (double)k / (double)(t + k));
        const uint64_t u = smix((uint64_t)t * 7 + 1);
        h[(size_t)t] = (int64_t)((uint64_t)INT64_MIN + (uint64_t)((double)(u >> 11) / 9007199254740992.0 * frac * span));
        rows[(size_t)(t * W)] = smix((uint64_t)t * 13 + 5);
        rows[(size_t)(t * W + 1)] = smix((uint64_t)t * 17 + 9);
    }
    for (int rep = 0; rep < 3; ++rep) {
        rsv::HostValuesWide a, b;
        a.reset(k, W);
        b.reset(k, W);
        auto t0 = std::chrono::steady_clock::now();
        for (int64_t t = 0; t < N; ++t) a.sample_first(h[(size_t)t], rows.data() + t * W);
        a.table_rebuild();
        auto t1 = std::chrono::steady_clock::now();
        for (int64_t t = 0; t < N; ++t) b.sample_first_at(h[(size_t)t], t);
        b.adopt(rows.data());
        b.table_rebuild();
        auto t2 = std::chrono::steady_clock::now();
        rsv::HostValues c;  // the Long replica's heap-only run over the same hashes (element = t)
        c.reset(k);
        std::vector<uint8_t> first((size_t)N, 1);
        auto t3 = std::chrono::steady_clock::now();
        c.sample_run_unique(N, first.data(), [](int64_t t) { return t; }, [&](int64_t t) { return h[(size_t)t]; });
        auto t4 = std::chrono::steady_clock::now();
        const double dc = std::chrono::duration<double, std::milli>(t4 - t3).count();
        std::printf("{\"long_heap_only_ms\": %.2f, \"ns_per_row\": %.1f}\n", dc, dc * 1e6 / N);
        std::vector<int64_t> ha, hb;
        std::vector<uint64_t> ra, rb;
        a.members_heap(ha, ra);
        b.members_heap(hb, rb);
        const double da = std::chrono::duration<double, std::milli>(t1 - t0).count();
        const double db = std::chrono::duration<double, std::milli>(t2 - t1).count();
        std::printf("{\"rows\": %lld, \"slot_copy_ms\": %.2f, \"log_pos_ms\": %.2f, \"ns_per_row\": [%.1f, %.1f], "
                    "\"identical\": %s, \"max_hash_equal\": %s}\n",
                    (long long)N, da, db, da * 1e6 / N, db * 1e6 / N, (ha == hb && ra == rb) ? "true" : "false",
                    a.max_hash == b.max_hash ? "true" : "false");
    }
    return 0;
}
