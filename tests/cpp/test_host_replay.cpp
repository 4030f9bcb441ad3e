// Host-only check of the ordered-distinct replica's two replay forms (rsv_host_values.h): the
// set-based run (RandomValues.sample per candidate, Sampler.scala:394-409) and the heap-only run
// over first-occurrence flags (the flags computed here on the host exactly as rsv_distinct.hip's
// mark_first defines them: the key neither occurs earlier in the segment nor is a member when the
// segment starts).  Both replicas consume the same segments; after every segment their heaps
// (hash and element arrays, size, maxHash) must be identical.  Set-based calls after a heap-only
// run (rebuild of the element set) are interleaved.  A third replica, HostValuesWide (the byte-key
// form of rsv_wide.hip) fed each key as the two-word row [key, ~key], must hold the same heap entry
// for entry (hash, and the row's first word = the key); a fourth, HostValuesWide fed only the flagged
// first occurrences through sample_first (heap only, its element table rebuilt afterwards -- the
// wide replay's first-occurrence form), too.  Exit 0 and "ok <cases>" on success.
//   g++ -std=c++17 -O2 -I reservoir_amd/csrc tests/cpp/test_host_replay.cpp -o test_host_replay
#include <cstdio>
#include <cstring>
#include <random>
#include <unordered_set>
#include <vector>

#include "rsv_host_values.h"

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static bool same(const rsv::HostValues& a, const rsv::HostValues& b) {
    if (a.n != b.n || a.max_hash != b.max_hash) return false;
    for (int64_t i = 1; i <= a.n; ++i)
        if (a.hh[(size_t)i] != b.hh[(size_t)i] || a.he[(size_t)i] != b.he[(size_t)i]) return false;
    return true;
}

static bool same_wide(const rsv::HostValues& a, const rsv::HostValuesWide& c) {
    if (a.n != c.n || a.max_hash != c.max_hash) return false;
    for (int64_t i = 1; i <= a.n; ++i) {
        const uint64_t* r = c.row(c.hs[(size_t)i]);
        if (a.hh[(size_t)i] != c.hh[(size_t)i] || (uint64_t)a.he[(size_t)i] != r[0] || r[1] != ~r[0]) return false;
    }
    return true;
}

int main() {
    int cases = 0;
    for (const int64_t k : {1, 2, 5, 64, 1000, 4096}) {
        for (const int64_t buckets : {3, 50, 100000}) {  // distinct hash values: ties at every size
            for (const uint64_t seed : {1ull, 2ull, 3ull}) {
                std::mt19937_64 rng(seed * 7919 + (uint64_t)k * 31 + (uint64_t)buckets);
                const int64_t universe = std::max<int64_t>(4, 6 * k);  // keys repeat across segments
                rsv::HostValues a, b;
                rsv::HostValuesWide cw, cf;
                a.reset(k);
                b.reset(k);
                cw.reset(k, 2);
                cf.reset(k, 2);
                for (int seg = 0; seg < 12; ++seg) {
                    const int64_t c = (int64_t)(rng() % (uint64_t)(3 * k + 50));
                    std::vector<int64_t> ek((size_t)c), eh((size_t)c);
                    for (int64_t t = 0; t < c; ++t) {
                        // a few keys equal to the set's free-slot sentinel exercise its side flag
                        const int64_t key = (rng() % 97 == 0) ? (int64_t)0x8000000000000001ull
                                                              : (int64_t)(rng() % (uint64_t)universe) - universe / 2;
                        ek[(size_t)t] = key;
                        eh[(size_t)t] = (int64_t)mix64((uint64_t)key % (uint64_t)buckets + 11) ;
                    }
                    for (int64_t t = 0; t < c; ++t) {
                        const uint64_t row[2] = {(uint64_t)ek[(size_t)t], ~(uint64_t)ek[(size_t)t]};
                        cw.sample(eh[(size_t)t], row);
                    }
                    if (seg % 4 == 3) {  // set-based single calls on both (b rebuilds its set)
                        for (int64_t t = 0; t < c; ++t) {
                            a.sample(ek[(size_t)t], eh[(size_t)t]);
                            b.sample(ek[(size_t)t], eh[(size_t)t]);
                            const uint64_t row[2] = {(uint64_t)ek[(size_t)t], ~(uint64_t)ek[(size_t)t]};
                            cf.sample(eh[(size_t)t], row);
                        }
                    } else {
                        std::unordered_set<int64_t> seen;
                        for (int64_t i = 1; i <= b.n; ++i) seen.insert(b.he[(size_t)i]);
                        std::vector<uint8_t> first((size_t)c);
                        for (int64_t t = 0; t < c; ++t) first[(size_t)t] = seen.insert(ek[(size_t)t]).second ? 1 : 0;
                        a.sample_run(c, [&](int64_t t) { return ek[(size_t)t]; }, [&](int64_t t) { return eh[(size_t)t]; });
                        b.sample_run_unique(c, first.data(), [&](int64_t t) { return ek[(size_t)t]; },
                                            [&](int64_t t) { return eh[(size_t)t]; });
                        for (int64_t t = 0; t < c; ++t) {
                            if (!first[(size_t)t]) continue;
                            const uint64_t row[2] = {(uint64_t)ek[(size_t)t], ~(uint64_t)ek[(size_t)t]};
                            cf.sample_first(eh[(size_t)t], row);
                        }
                        cf.table_rebuild();
                    }
                    if (!same(a, b) || !same_wide(a, cw) || !same_wide(a, cf)) {
                        std::printf("MISMATCH k=%lld buckets=%lld seed=%llu segment=%d\n", (long long)k,
                                    (long long)buckets, (unsigned long long)seed, seg);
                        return 1;
                    }
                    ++cases;
                }
            }
        }
    }
    std::printf("ok %d\n", cases);
    return 0;
}
