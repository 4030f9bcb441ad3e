// micro_heap.cpp -- host replay cost of RSV_DISTINCT_ORDERED (development probe, not part of the
// library): the scala-PriorityQueue replica's replace step (dequeue + enqueue, Sampler.scala:403-407)
// on a synthetic accepted-candidate stream (each accepted h uniform below the current maximum, as
// in a long stream), branchy vs branch-free child selection; then the library's own replica
// (rsv_host_values.h, included as is) replaying chunk-filtered survivors of a C4-like stream against
// a branchy restatement of the same replica.  Both variants must leave identical heaps (checked).
//   g++ -O3 -march=native -std=c++17 tools/micro_heap.cpp -o /tmp/micro_heap && /tmp/micro_heap
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../reservoir_amd/csrc/rsv_host_values.h"

struct Branchy {  // as HostValues (rsv_distinct.hip) before this probe: vector-backed, bounds-tested
    std::vector<int64_t> hh{0}, he{0};
    int64_t size() const { return (int64_t)hh.size() - 1; }
    void add(int64_t e, int64_t h) {
        hh.push_back(h);
        he.push_back(e);
        size_t m = hh.size() - 1;
        while (m > 1 && hh[m / 2] < h) {
            hh[m] = hh[m / 2];
            he[m] = he[m / 2];
            m /= 2;
        }
        hh[m] = h;
        he[m] = e;
    }
    int64_t dequeue() {
        const int64_t res = he[1];
        const int64_t h = hh.back(), e = he.back();
        hh.pop_back();
        he.pop_back();
        const int64_t n = size();
        if (n == 0) return res;
        int64_t kk = 1;
        while (n >= 2 * kk) {
            int64_t j = 2 * kk;
            if (j < n && hh[j] < hh[j + 1]) ++j;
            if (h >= hh[j]) break;
            hh[kk] = hh[j];
            he[kk] = he[j];
            kk = j;
        }
        hh[kk] = h;
        he[kk] = e;
        return res;
    }
};

struct Flat {  // fixed arrays, explicit size, branch-free child choice, one slot of slack
    std::vector<int64_t> hh, he;
    int64_t n = 0;
    explicit Flat(int64_t cap) : hh((size_t)cap + 2, INT64_MIN), he((size_t)cap + 2, 0) {}
    void add(int64_t e, int64_t h) {
        int64_t m = ++n;
        int64_t* H = hh.data();
        int64_t* E = he.data();
        while (m > 1 && H[m >> 1] < h) {
            H[m] = H[m >> 1];
            E[m] = E[m >> 1];
            m >>= 1;
        }
        H[m] = h;
        E[m] = e;
    }
    int64_t dequeue() {
        int64_t* H = hh.data();
        int64_t* E = he.data();
        const int64_t res = E[1];
        const int64_t h = H[n], e = E[n];
        const int64_t nn = --n;
        if (nn == 0) return res;
        H[nn + 1] = h;  // slack slot: a right child past the end compares as the sinking entry
        int64_t kk = 1;
        while (nn >= 2 * kk) {
            int64_t j = 2 * kk;
            __builtin_prefetch(&H[4 * j]);
            j += H[j] < H[j + 1];
            if (h >= H[j]) break;
            H[kk] = H[j];
            E[kk] = E[j];
            kk = j;
        }
        H[kk] = h;
        E[kk] = e;
        return res;
    }
};

template <class Q>
static double run(Q& q, int64_t k, int64_t steps, uint64_t seed, int64_t* checksum) {
    std::mt19937_64 rng(seed);
    for (int64_t i = 0; i < k; ++i) q.add(i, (int64_t)rng());
    int64_t mx = 0;
    const auto t0 = std::chrono::steady_clock::now();
    int64_t cs = 0;
    for (int64_t s = 0; s < steps; ++s) {
        // accepted candidate: uniform below the current maximum
        // (head of the heap; both variants keep it at index 1)
        const int64_t top = q.hh[1];
        const uint64_t span = (uint64_t)top - (uint64_t)INT64_MIN;
        const int64_t h = (int64_t)((uint64_t)INT64_MIN + (span ? rng() % span : 0));
        cs += q.dequeue();
        q.add(k + s, h);
        mx = q.hh[1];
    }
    const auto t1 = std::chrono::steady_clock::now();
    *checksum = cs ^ mx;
    return std::chrono::duration<double>(t1 - t0).count();
}

// The replica as it was before rsv_host_values.h: branchy vector-backed heap + the same
// open-addressing set (borrowed from the library's struct, heap unused)
struct OldReplica {
    Branchy q;
    rsv::HostValues sv;
    int64_t k, max_hash = INT64_MIN;
    explicit OldReplica(int64_t kk) : k(kk) { sv.reset(kk); }
    void sample(int64_t e, int64_t h) {
        if (q.size() < k) {
            if (!sv.contains(e)) {
                if (q.size() + 1 > (int64_t)(sv.mask + 1) / 2 - 1) sv.set_reserve(2 * q.size() + 2);
                q.add(e, h);
                sv.set_add(e);
                if (h > max_hash) max_hash = h;
            }
        } else if (h < max_hash && !sv.contains(e)) {
            sv.set_remove(q.dequeue());
            q.add(e, h);
            sv.set_add(e);
            max_hash = q.hh[1];
        }
    }
};

static uint64_t scramble(uint64_t z) {  // stands in for the scrambled hash: any well-mixed 64-bit map
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// C4-like stream (30 % duplicates) cut into doubling chunks; per chunk the survivors of the
// GPU filter (all while not full, else h < maxHash at the chunk start) are replayed in order.
template <class R, class Replay>
static double replay_stream(R& r, int64_t n, int64_t k, Replay replay, int64_t* survivors) {
    std::vector<int64_t> ck, chh;
    int64_t pos = 0, seen = 0;
    double t = 0;
    *survivors = 0;
    while (pos < n) {
        const bool full = r.size() == k;
        const int64_t m = std::min<int64_t>(n - pos, full ? std::max<int64_t>(seen, 65536) : 2 * (k - r.size()) + 1024);
        const int64_t mh = r.max_hash;
        ck.clear();
        chh.clear();
        for (int64_t i = pos; i < pos + m; ++i) {
            const int64_t key = (int64_t)(scramble((uint64_t)i * 7 + 1) % (uint64_t)(n * 7 / 10));
            const int64_t h = (int64_t)scramble((uint64_t)key ^ 0x5DEECE66Dull);
            if (!full || h < mh) {
                ck.push_back(key);
                chh.push_back(h);
            }
        }
        *survivors += (int64_t)ck.size();
        const auto t0 = std::chrono::steady_clock::now();
        replay(r, ck, chh);
        t += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        pos += m;
        seen += m;
    }
    return t;
}

struct NewAdapter {
    rsv::HostValues v;
    int64_t max_hash = 0;
    int64_t size() const { return v.size(); }
};

int main() {
    const int64_t k = 65536, steps = 600000;
    for (int rep = 0; rep < 3; ++rep) {
        Branchy a;
        Flat b(k);
        int64_t ca = 0, cb = 0;
        const double ta = run(a, k, steps, 7 + rep, &ca);
        const double tb = run(b, k, steps, 7 + rep, &cb);
        bool same = ca == cb && std::memcmp(a.hh.data() + 1, b.hh.data() + 1, k * 8) == 0 &&
                    std::memcmp(a.he.data() + 1, b.he.data() + 1, k * 8) == 0;
        std::printf("replace step: branchy %.1f ns/step  flat %.1f ns/step  identical=%d\n", ta / steps * 1e9,
                    tb / steps * 1e9, (int)same);
    }
    const int64_t n = 100000000;
    OldReplica o(k);
    int64_t so = 0, sn = 0;
    struct OldView {  // what the chunk sizing reads: size() and max_hash at the chunk start
        OldReplica* o;
        int64_t size() const { return o->q.size(); }
        int64_t max_hash;
    };
    OldView ov{&o, o.max_hash};
    const double to = replay_stream(ov, n, k,
                                    [&](OldView& v, const std::vector<int64_t>& ck, const std::vector<int64_t>& ch) {
                                        for (size_t t = 0; t < ck.size(); ++t) v.o->sample(ck[t], ch[t]);
                                        v.max_hash = v.o->max_hash;
                                    },
                                    &so);
    NewAdapter na;
    na.v.reset(k);
    na.max_hash = na.v.max_hash;
    const double tn = replay_stream(na, n, k,
                                    [&](NewAdapter& v, const std::vector<int64_t>& ck, const std::vector<int64_t>& ch) {
                                        v.v.sample_run((int64_t)ck.size(), [&](int64_t t) { return ck[(size_t)t]; },
                                                       [&](int64_t t) { return ch[(size_t)t]; });
                                        v.max_hash = v.v.max_hash;
                                    },
                                    &sn);
    bool same = so == sn && o.q.size() == na.v.size() && o.max_hash == na.v.max_hash;
    for (int64_t i = 1; same && i <= k; ++i) same = o.q.hh[(size_t)i] == na.v.hh[(size_t)i] && o.q.he[(size_t)i] == na.v.he[(size_t)i];
    std::printf("replica over %lld elements (%lld survivors): old %.1f ms  library %.1f ms  identical=%d\n",
                (long long)n, (long long)sn, to * 1e3, tn * 1e3, (int)same);
    return same ? 0 : 1;
}
