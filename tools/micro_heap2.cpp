// micro_heap2.cpp -- development probe (not part of the library): the full-heap phase of the
// ordered-distinct host replay (Sampler.scala:403-407) on one recorded candidate log, with variants
// of the replica.  Every variant must leave the heap identical to rsv_host_values.h's (checked).
//   g++ -O3 -march=native -std=c++17 tools/micro_heap2.cpp -o /tmp/micro_heap2 && /tmp/micro_heap2
// On the MI355X box's host (EPYC 9575F, 5e8-element stream, 995k-entry log, 585k replacements):
// set-based library replica 36.8-38.7 ms; heap only 23.2 (+ deep prefetch 22.7); look-ahead 2/3
// levels 23.5/28.0; bottom-up 31.5; branch-free descent 31.9; huge pages 22.4-22.7; a seen-set
// instead of the member set 42.7.  The product took heap only + deep prefetch (rsv_host_values.h).
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include <sys/mman.h>
#include <cstdlib>

#include "../reservoir_amd/csrc/rsv_host_values.h"

static uint64_t scramble(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// heap-only replica: the log holds first occurrences only (no set probes)
template <int PF>
struct HeapOnly {
    std::vector<int64_t> hh, he;
    int64_t k, n = 0, max_hash = INT64_MIN;
    explicit HeapOnly(int64_t kk) : hh((size_t)kk + 2, INT64_MIN), he((size_t)kk + 2, 0), k(kk) {}
    void add(int64_t e, int64_t h) {
        int64_t* H = hh.data();
        int64_t* E = he.data();
        int64_t m = ++n;
        while (m > 1 && H[m >> 1] < h) {
            H[m] = H[m >> 1];
            E[m] = E[m >> 1];
            m >>= 1;
        }
        H[m] = h;
        E[m] = e;
    }
    void dequeue() {
        int64_t* H = hh.data();
        int64_t* E = he.data();
        const int64_t h = H[n], e = E[n];
        const int64_t nn = --n;
        H[nn + 1] = h;
        const int64_t last = (int64_t)hh.size() - 1;
        int64_t kk = 1;
        while (nn >= 2 * kk) {
            int64_t j = 2 * kk;
            if (PF >= 1) __builtin_prefetch(H + std::min(4 * j, last));
            if (PF >= 2) {
                __builtin_prefetch(H + std::min(8 * j, last));
                __builtin_prefetch(H + std::min(8 * j + 8, last));
            }
            if (PF >= 3) {
                __builtin_prefetch(E + std::min(2 * j, last));
            }
            j += H[j] < H[j + 1];
            if (h >= H[j]) break;
            H[kk] = H[j];
            E[kk] = E[j];
            kk = j;
        }
        H[kk] = h;
        E[kk] = e;
    }
    void run(int64_t c, const int64_t* ek, const int64_t* eh) {
        int64_t t = 0;
        for (; t < c && n < k; ++t) {
            add(ek[t], eh[t]);
            if (eh[t] > max_hash) max_hash = eh[t];
        }
        for (; t < c; ++t) {
            const int64_t h = eh[t];
            if (h < max_hash) {
                dequeue();
                add(ek[t], h);
                max_hash = hh[1];
            }
        }
    }
};

// heap-only, bottom-up fixDown: the larger-child path to the bottom, then the sinking entry's place
// found climbing back (the path's hashes only fall, so the first place from the top where
// h >= H[path] is where the standard fixDown stops)
struct BottomUp : HeapOnly<1> {
    using HeapOnly<1>::HeapOnly;
    void dequeue() {
        int64_t* H = hh.data();
        int64_t* E = he.data();
        const int64_t h = H[n], e = E[n];
        const int64_t nn = --n;
        H[nn + 1] = h;
        const int64_t last = (int64_t)hh.size() - 1;
        int64_t j = 1;
        while (nn >= 2 * j) {
            int64_t c = 2 * j;
            __builtin_prefetch(H + std::min(4 * c, last));
            c += H[c] < H[c + 1];
            j = c;
        }
        // j is the bottom of the path; climb while h >= H[j] (i.e. the standard loop would stop above j)
        while (j > 1 && h >= H[j]) j >>= 1;
        // shift the path [1 .. j] up one level
        const int d = 63 - __builtin_clzll((uint64_t)j);
        int64_t kk = 1;
        for (int s = d - 1; s >= 0; --s) {
            const int64_t c = j >> s;
            H[kk] = H[c];
            E[kk] = E[c];
            kk = c;
        }
        H[kk] = h;
        E[kk] = e;
    }
    void run(int64_t c, const int64_t* ek, const int64_t* eh) {
        int64_t t = 0;
        for (; t < c && n < k; ++t) {
            add(ek[t], eh[t]);
            if (eh[t] > max_hash) max_hash = eh[t];
        }
        for (; t < c; ++t) {
            const int64_t h = eh[t];
            if (h < max_hash) {
                dequeue();
                add(ek[t], h);
                max_hash = hh[1];
            }
        }
    }
};

// heap-only, two levels per step: the children and all four grandchildren are loaded from kk alone,
// so the per-level dependence is a compare + select instead of a load
template <int L>
struct Ahead : HeapOnly<0> {
    explicit Ahead(int64_t kk) : HeapOnly<0>(kk) {
        hh.resize((size_t)(8 * kk + 16), INT64_MIN);
        he.resize(hh.size(), 0);
    }
    void dequeue() {
        int64_t* H = hh.data();
        int64_t* E = he.data();
        const int64_t h = H[n], e = E[n];
        const int64_t nn = --n;
        H[nn + 1] = h;
        int64_t kk = 1;
        for (;;) {
            int64_t j = 2 * kk;
            if (nn < j) break;
            const int64_t a = H[j], b = H[j + 1];
            const int64_t q0 = H[2 * j], q1 = H[2 * j + 1], q2 = H[2 * j + 2], q3 = H[2 * j + 3];
            int64_t r[8];
            if (L == 3)
                for (int i = 0; i < 8; ++i) r[i] = H[4 * j + i];
            const int s = a < b;
            const int64_t hj = s ? b : a;
            j += s;
            if (h >= hj) break;
            H[kk] = hj;
            E[kk] = E[j];
            kk = j;
            int64_t j2 = 2 * kk;
            if (nn < j2) break;
            const int64_t c0 = s ? q2 : q0, c1 = s ? q3 : q1;
            const int s2 = c0 < c1;
            const int64_t hc = s2 ? c1 : c0;
            j2 += s2;
            if (h >= hc) break;
            H[kk] = hc;
            E[kk] = E[j2];
            kk = j2;
            if (L == 3) {
                int64_t j3 = 2 * kk;
                if (nn < j3) break;
                const int o = 4 * s + 2 * s2;
                const int64_t d0 = r[o], d1 = r[o + 1];
                const int s3 = d0 < d1;
                const int64_t hd = s3 ? d1 : d0;
                j3 += s3;
                if (h >= hd) break;
                H[kk] = hd;
                E[kk] = E[j3];
                kk = j3;
            }
        }
        H[kk] = h;
        E[kk] = e;
    }
    void run(int64_t c, const int64_t* ek, const int64_t* eh) {
        int64_t t = 0;
        for (; t < c && n < k; ++t) {
            add(ek[t], eh[t]);
            if (eh[t] > max_hash) max_hash = eh[t];
        }
        for (; t < c; ++t) {
            const int64_t h = eh[t];
            if (h < max_hash) {
                dequeue();
                add(ek[t], h);
                max_hash = hh[1];
            }
        }
    }
};

// "seen" set instead of the member set: only the first occurrence of a key can ever be admitted
// (a repeat of a member fails contains; of an evicted or rejected key fails h < maxHash, maxHash
// never rises once full), so the set need not drop evicted keys: it must hold every member, and
// may hold any key whose hash is above the current maxHash.  One probe per candidate (find or
// insert); entries {key, h}; when the table passes half full it is rebuilt keeping h <= maxHash.
struct SeenSet {
    std::vector<int64_t> sk, sh;
    uint64_t mask = 0;
    int64_t cnt = 0;
    static constexpr int64_t kEmpty = (int64_t)0x8000000000000001ull;
    bool has_empty = false;
    static uint64_t mix(int64_t v) {
        uint64_t z = (uint64_t)v * 0x9E3779B97F4A7C15ull;
        return z ^ (z >> 29);
    }
    void init(uint64_t cap) {
        sk.assign(cap, kEmpty);
        sh.assign(cap, 0);
        mask = cap - 1;
        cnt = 0;
    }
    // true when v was not present (and is now)
    bool insert(int64_t v, int64_t h) {
        if (v == kEmpty) {
            const bool fresh = !has_empty;
            has_empty = true;
            return fresh;
        }
        uint64_t q = mix(v) & mask;
        for (;; q = (q + 1) & mask) {
            const int64_t s = sk[q];
            if (s == v) return false;
            if (s == kEmpty) break;
        }
        sk[q] = v;
        sh[q] = h;
        ++cnt;
        return true;
    }
    void prefetch(int64_t v) const { __builtin_prefetch(&sk[mix(v) & mask]); }
    void prune(int64_t max_h) {  // keep keys with h <= max_h
        std::vector<int64_t> ok, oh;
        ok.swap(sk);
        oh.swap(sh);
        init(ok.size());
        for (size_t i = 0; i < ok.size(); ++i)
            if (ok[i] != kEmpty && oh[i] <= max_h) insert(ok[i], oh[i]);
    }
};

struct SeenReplica : HeapOnly<1> {
    SeenSet seen;
    explicit SeenReplica(int64_t kk) : HeapOnly<1>(kk) { seen.init(1u << 18); }
    void run(int64_t c, const int64_t* ek, const int64_t* eh) {
        int64_t t = 0;
        for (; t < c && n < k; ++t)
            if (seen.insert(ek[t], eh[t])) {
                add(ek[t], eh[t]);
                if (eh[t] > max_hash) max_hash = eh[t];
            }
        constexpr int64_t kAhead = 8;
        for (int64_t p = t; p < std::min(c, t + kAhead); ++p)
            if (eh[p] < max_hash) seen.prefetch(ek[p]);
        for (; t < c; ++t) {
            const int64_t p = t + kAhead;
            if (p < c && eh[p] < max_hash) seen.prefetch(ek[p]);
            const int64_t h = eh[t];
            if (h < max_hash && seen.insert(ek[t], h)) {
                dequeue();
                add(ek[t], h);
                max_hash = hh[1];
                if (seen.cnt * 2 > (int64_t)seen.mask) seen.prune(max_hash);
            }
        }
    }
};

// heap-only, branch-free fixDown: the larger-child path (left on ties) to the last complete level
// (plus one step into a partial level), the moves counted as the path entries above the sinking
// hash (the path's hashes only fall), every path node rewritten with a selected value
struct Branchless : HeapOnly<0> {
    using HeapOnly<0>::HeapOnly;
    void dequeue() {
        int64_t* H = hh.data();
        int64_t* E = he.data();
        const int64_t h = H[n], e = E[n];
        const int64_t nn = --n;
        if (nn == 0) return;
        H[nn + 1] = h;
        const int L = 63 - __builtin_clzll((uint64_t)nn + 1);  // complete levels
        int64_t pp[64], pv[64];
        int64_t p = 1;
        int D = L - 1;
        for (int d = 0; d < D; ++d) {
            int64_t c = 2 * p;
            const int64_t a = H[c], b = H[c + 1];
            const bool s = a < b;
            c += s;
            pv[d] = s ? b : a;
            pp[d] = c;
            p = c;
        }
        if (2 * p <= nn) {
            int64_t c = 2 * p;
            const int64_t a = H[c], b = H[c + 1];
            const bool s = a < b;
            c += s;
            pv[D] = s ? b : a;
            pp[D] = c;
            ++D;
        }
        int m = 0;
        for (int d = 0; d < D; ++d) m += pv[d] > h;
        // moves: node_d (node_0 = 1, node_{d+1} = pp[d]) takes the entry of node_{d+1} for d < m;
        // node_m takes the sinking entry
        int64_t node = 1;
        for (int d = 0; d < m; ++d) {
            H[node] = pv[d];
            E[node] = E[pp[d]];
            node = pp[d];
        }
        H[node] = h;
        E[node] = e;
    }
    void run(int64_t c, const int64_t* ek, const int64_t* eh) {
        int64_t t = 0;
        for (; t < c && n < k; ++t) {
            add(ek[t], eh[t]);
            if (eh[t] > max_hash) max_hash = eh[t];
        }
        for (; t < c; ++t) {
            const int64_t h = eh[t];
            if (h < max_hash) {
                dequeue();
                add(ek[t], h);
                max_hash = hh[1];
            }
        }
    }
};

// heap-only over arrays in one 2 MB-aligned block advised as a huge page (the deep levels' lines are
// on 128 different 4 KB pages otherwise)
template <int PF>
struct HugeHeap {
    int64_t* H;
    int64_t* E;
    int64_t k, n = 0, max_hash = INT64_MIN, cap;
    std::vector<int64_t> hh, he;  // copies for the check
    explicit HugeHeap(int64_t kk) : k(kk) {
        cap = ((kk + 2) * 8 + (2 << 20) - 1) / (2 << 20) * (2 << 20);
        void* m = std::aligned_alloc(2 << 20, 2 * cap);
        madvise(m, 2 * cap, MADV_HUGEPAGE);
        std::memset(m, 0, 2 * cap);
        H = (int64_t*)m;
        E = (int64_t*)((char*)m + cap);
    }
    void add(int64_t e, int64_t h) {
        int64_t m = ++n;
        while (m > 1 && H[m >> 1] < h) {
            H[m] = H[m >> 1];
            E[m] = E[m >> 1];
            m >>= 1;
        }
        H[m] = h;
        E[m] = e;
    }
    void dequeue() {
        const int64_t h = H[n], e = E[n];
        const int64_t nn = --n;
        H[nn + 1] = h;
        const int64_t last = cap / 8 - 1;
        int64_t kk = 1;
        while (nn >= 2 * kk) {
            int64_t j = 2 * kk;
            __builtin_prefetch(H + std::min(4 * j, last));
            if (PF >= 2) {
                __builtin_prefetch(H + std::min(8 * j, last));
                __builtin_prefetch(H + std::min(8 * j + 8, last));
            }
            j += H[j] < H[j + 1];
            if (h >= H[j]) break;
            H[kk] = H[j];
            E[kk] = E[j];
            kk = j;
        }
        H[kk] = h;
        E[kk] = e;
    }
    void run(int64_t c, const int64_t* ek, const int64_t* eh) {
        int64_t t = 0;
        for (; t < c && n < k; ++t) {
            add(ek[t], eh[t]);
            if (eh[t] > max_hash) max_hash = eh[t];
        }
        for (; t < c; ++t) {
            const int64_t h = eh[t];
            if (h < max_hash) {
                dequeue();
                add(ek[t], h);
                max_hash = H[1];
            }
        }
        hh.assign(H, H + k + 2);
        he.assign(E, E + k + 2);
    }
};

// heap-only (+ deep prefetch) with the admission test taken a block of 64 entries at a time against
// the block's starting maxHash (branch-free selection), then re-tested exactly per selected entry
// (maxHash only falls within the block, so the re-test mostly passes: a predictable branch)
struct Blocked : HeapOnly<2> {
    using HeapOnly<2>::HeapOnly;
    void run(int64_t c, const int64_t* ek, const int64_t* eh) {
        int64_t t = 0;
        for (; t < c && n < k; ++t) {
            add(ek[t], eh[t]);
            if (eh[t] > max_hash) max_hash = eh[t];
        }
        uint32_t sel[64];
        while (t < c) {
            const int64_t e = std::min<int64_t>(c, t + 64);
            const int64_t mh = max_hash;
            int cnt = 0;
            for (int64_t u = t; u < e; ++u) {
                sel[cnt] = (uint32_t)(u - t);
                cnt += eh[u] < mh;
            }
            for (int i = 0; i < cnt; ++i) {
                const int64_t u = t + sel[i];
                const int64_t h = eh[u];
                if (h < max_hash) {
                    dequeue();
                    add(ek[u], h);
                    max_hash = hh[1];
                }
            }
            t = e;
        }
    }
};

// heap-only with each node's (hash, element) side by side (one 16-B slot): a level's move reads the
// element from the line its hash came in (one line per level instead of two)
template <int PF>
struct Aos {
    struct Node {
        int64_t h, e;
    };
    std::vector<Node> a;
    int64_t k, n = 0, max_hash = INT64_MIN;
    std::vector<int64_t> hh, he;  // copies for the check
    explicit Aos(int64_t kk) : a((size_t)(8 * kk + 16), Node{INT64_MIN, 0}), k(kk) {}
    void add(int64_t e, int64_t h) {
        Node* A = a.data();
        int64_t m = ++n;
        while (m > 1 && A[m >> 1].h < h) {
            A[m] = A[m >> 1];
            m >>= 1;
        }
        A[m] = Node{h, e};
    }
    void dequeue() {
        Node* A = a.data();
        const Node x = A[n];
        const int64_t nn = --n;
        A[nn + 1].h = x.h;
        int64_t kk = 1;
        while (nn >= 2 * kk) {
            int64_t j = 2 * kk;
            if (PF >= 1) __builtin_prefetch(A + 4 * j);
            if (PF >= 2) __builtin_prefetch(A + 4 * j + 4);
            j += A[j].h < A[j + 1].h;
            if (x.h >= A[j].h) break;
            A[kk] = A[j];
            kk = j;
        }
        A[kk] = x;
    }
    void run(int64_t c, const int64_t* ek, const int64_t* eh) {
        int64_t t = 0;
        for (; t < c && n < k; ++t) {
            add(ek[t], eh[t]);
            if (eh[t] > max_hash) max_hash = eh[t];
        }
        for (; t < c; ++t) {
            const int64_t h = eh[t];
            if (h < max_hash) {
                dequeue();
                add(ek[t], h);
                max_hash = a[1].h;
            }
        }
        hh.resize((size_t)k + 2);
        he.resize((size_t)k + 2);
        for (int64_t i = 1; i <= k; ++i) hh[i] = a[i].h, he[i] = a[i].e;
    }
};

// heap-only with 4-byte element slots (the entry's log position; the key is read from the log at
// the end): the element array is half the bytes, so the hashes + elements fit the core's L2 better
template <int PF>
struct Idx32 {
    std::vector<int64_t> hh, he;
    std::vector<uint32_t> ei;
    int64_t k, n = 0, max_hash = INT64_MIN;
    explicit Idx32(int64_t kk) : hh((size_t)kk + 2, INT64_MIN), ei((size_t)kk + 2, 0), k(kk) {}
    void add(uint32_t e, int64_t h) {
        int64_t* H = hh.data();
        uint32_t* E = ei.data();
        int64_t m = ++n;
        while (m > 1 && H[m >> 1] < h) {
            H[m] = H[m >> 1];
            E[m] = E[m >> 1];
            m >>= 1;
        }
        H[m] = h;
        E[m] = e;
    }
    void dequeue() {
        int64_t* H = hh.data();
        uint32_t* E = ei.data();
        const int64_t h = H[n];
        const uint32_t e = E[n];
        const int64_t nn = --n;
        H[nn + 1] = h;
        const int64_t last = (int64_t)hh.size() - 1;
        int64_t kk = 1;
        while (nn >= 2 * kk) {
            int64_t j = 2 * kk;
            if (PF >= 1) __builtin_prefetch(H + std::min(4 * j, last));
            if (PF >= 2) {
                __builtin_prefetch(H + std::min(8 * j, last));
                __builtin_prefetch(H + std::min(8 * j + 8, last));
            }
            j += H[j] < H[j + 1];
            if (h >= H[j]) break;
            H[kk] = H[j];
            E[kk] = E[j];
            kk = j;
        }
        H[kk] = h;
        E[kk] = e;
    }
    void run(int64_t c, const int64_t* ek, const int64_t* eh) {
        int64_t t = 0;
        for (; t < c && n < k; ++t) {
            add((uint32_t)t, eh[t]);
            if (eh[t] > max_hash) max_hash = eh[t];
        }
        for (; t < c; ++t) {
            const int64_t h = eh[t];
            if (h < max_hash) {
                dequeue();
                add((uint32_t)t, h);
                max_hash = hh[1];
            }
        }
        he.resize((size_t)k + 2);
        for (int64_t i = 1; i <= k; ++i) he[i] = ek[ei[i]];
    }
};

template <class F>
static double timed(F f) {
    const auto t0 = std::chrono::steady_clock::now();
    f();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3;
}

int main(int argc, char** argv) {
    const int64_t k = argc > 2 ? atoll(argv[2]) : 65536, n = argc > 1 ? atoll(argv[1]) : 300000000;
    const double beta = 1.6;
    // the log: distinct keys; while not full everything, then h below beta x the expected k-th
    // smallest hash at that position (a scheduled pass's superset)
    std::vector<int64_t> lk, lh;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t key = (int64_t)scramble((uint64_t)i * 0x9E3779B97F4A7C15ull + 11);
        const int64_t h = (int64_t)scramble((uint64_t)key ^ 0x5DEECE66Dull);
        if (i < 2 * k) {
            lk.push_back(key), lh.push_back(h);
            continue;
        }
        const double frac = beta * (double)k / (double)i;  // fraction of the hash range admitted
        const double bound = -9.223372036854775808e18 + frac * 1.8446744073709551616e19;
        if ((double)h < bound) lk.push_back(key), lh.push_back(h);
    }
    const int64_t c = (int64_t)lk.size();
    int64_t reps = 0;
    {
        HeapOnly<0> z(k);
        int64_t t = 0;
        for (; t < c && z.n < k; ++t) z.add(lk[t], lh[t]), z.max_hash = std::max(z.max_hash, lh[t]);
        for (; t < c; ++t)
            if (lh[t] < z.max_hash) z.dequeue(), z.add(lk[t], lh[t]), z.max_hash = z.hh[1], ++reps;
    }
    std::printf("n=%lld k=%lld log=%lld replacements=%lld\n", (long long)n, (long long)k, (long long)c, (long long)reps);
    for (int rep = 0; rep < 2; ++rep) {
        rsv::HostValues ref;
        ref.reset(k);
        const double t0 = timed([&] { ref.sample_run(c, [&](int64_t t) { return lk[t]; }, [&](int64_t t) { return lh[t]; }); });
        auto check = [&](const std::vector<int64_t>& H, const std::vector<int64_t>& E) {
            return std::memcmp(H.data() + 1, ref.hh.data() + 1, k * 8) == 0 &&
                   std::memcmp(E.data() + 1, ref.he.data() + 1, k * 8) == 0;
        };
        HeapOnly<1> a(k);
        const double t1 = timed([&] { a.run(c, lk.data(), lh.data()); });
        HeapOnly<2> b(k);
        const double t2 = timed([&] { b.run(c, lk.data(), lh.data()); });
        HeapOnly<3> b3(k);
        const double t3 = timed([&] { b3.run(c, lk.data(), lh.data()); });
        BottomUp u(k);
        const double t4 = timed([&] { u.run(c, lk.data(), lh.data()); });
        Ahead<2> w2(k);
        const double t5 = timed([&] { w2.run(c, lk.data(), lh.data()); });
        Ahead<3> w3(k);
        const double t6 = timed([&] { w3.run(c, lk.data(), lh.data()); });
        SeenReplica sr(k);
        const double t7 = timed([&] { sr.run(c, lk.data(), lh.data()); });
        Blocked bk(k);
        const double t11 = timed([&] { bk.run(c, lk.data(), lh.data()); });
        HeapOnly<2> b2(k);
        const double t12 = timed([&] { b2.run(c, lk.data(), lh.data()); });
        std::printf("blocked admission %.1f (%d) vs heap-only+deep %.1f\n", t11, (int)check(bk.hh, bk.he), t12);
        HugeHeap<1> hg1(k);
        const double t9 = timed([&] { hg1.run(c, lk.data(), lh.data()); });
        HugeHeap<2> hg2(k);
        const double t10 = timed([&] { hg2.run(c, lk.data(), lh.data()); });
        std::printf("huge page %.1f (%d) +deep prefetch %.1f (%d)\n", t9, (int)check(hg1.hh, hg1.he), t10,
                    (int)check(hg2.hh, hg2.he));
        Aos<1> o1(k);
        const double to1 = timed([&] { o1.run(c, lk.data(), lh.data()); });
        Aos<2> o2(k);
        const double to2 = timed([&] { o2.run(c, lk.data(), lh.data()); });
        Idx32<1> i1(k);
        const double ti1 = timed([&] { i1.run(c, lk.data(), lh.data()); });
        Idx32<2> i2(k);
        const double ti2 = timed([&] { i2.run(c, lk.data(), lh.data()); });
        std::printf("aos+pf %.1f (%d) aos+pf2 %.1f (%d) | idx32+pf %.1f (%d) idx32+deep %.1f (%d)\n", to1,
                    (int)check(o1.hh, o1.he), to2, (int)check(o2.hh, o2.he), ti1, (int)check(i1.hh, i1.he), ti2,
                    (int)check(i2.hh, i2.he));
        Branchless bl(k);
        const double t8 = timed([&] { bl.run(c, lk.data(), lh.data()); });
        std::printf("branchless descent %.1f (%d)\n", t8, (int)check(bl.hh, bl.he));
        std::printf("seen-set replica %.1f (%d)\n", t7, (int)check(sr.hh, sr.he));
        std::printf("ahead2 %.1f (%d) ahead3 %.1f (%d)\n", t5, (int)check(w2.hh, w2.he), t6, (int)check(w3.hh, w3.he));
        std::printf("library %.1f ms | heap-only %.1f (%d) | +deep prefetch %.1f (%d) | +E prefetch %.1f (%d) | bottom-up %.1f (%d)\n",
                    t0, t1, (int)check(a.hh, a.he), t2, (int)check(b.hh, b.he), t3, (int)check(b3.hh, b3.he), t4,
                    (int)check(u.hh, u.he));
    }
    return 0;
}
