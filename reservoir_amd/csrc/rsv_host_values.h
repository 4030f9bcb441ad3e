// rsv_host_values.h -- exact host replica of the reference's RandomValues state
// (Sampler.scala:389-409), used by RSV_DISTINCT_ORDERED to replay the GPU-filtered survivors of
// each chunk in arrival order.  Host-only C++ (no HIP): tools/micro_heap.cpp includes it as is.
//
// State: a 1-indexed binary max-heap on the hash with scala 2.13 mutable.PriorityQueue's tie
// behaviour (addOne/fixUp: sift up while parent < child; dequeue/fixDown: last entry to the root,
// sift down to the larger child -- left on ties -- and stop when parent >= child), an
// open-addressing element set, and maxHash.  (Product implementation; the oracle under oracle/ is
// an independent restatement for the tests.)
//
// Layout for the replay loop (~k ln(n/k) replace steps, inherently sequential): the heap lives in
// two flat arrays (hashes / elements, the sift loops compare hashes only; up to k + 2 entries) with
// an explicit size; the slot past the last entry holds the sinking hash during fixDown, so the child
// choice is one branch-free compare (`j += H[j] < H[j+1]`): a missing right child then equals the
// sinking entry, which never wins over a left child that is larger (same result as the bounds
// test it replaces).  The element set keeps one int64 per slot (a sentinel marks free slots).
// tools/micro_heap.cpp (identical heaps): replace step 143 -> 75 ns at k = 65536; whole replica
// over a C4-like 1e8-element stream (805k survivors) ~1.5x faster than the vector-backed branchy
// heap + 16-B set slots; C4 ordered end to end on MI355X 62.7 -> 50.9 ms.  A heap of (hash,
// element) pairs (one line per level) measured no better than the two arrays.
//
// Only the first occurrence of a key can ever be admitted: a repeat of a member fails contains, and
// a repeat of an evicted or rejected key fails h < maxHash (maxHash never rises once the heap is
// full; an evicted key had h = maxHash when it left).  So a run whose entries are marked "first
// occurrence since the run began, and not a member when it began" (computed on the device,
// rsv_distinct.hip: segment_first_flags) needs no set at all: sample_run_unique runs the heap
// alone, and the member set is rebuilt from the heap only if a set-based call comes later.
// tools/micro_heap2.cpp on the MI355X box's host (EPYC 9575F), 585k replacements at k = 65536:
// set-based 38.5 ms, heap only 23.6 ms (identical heaps).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rsv {

struct HostValues {
    struct Ent {
        int64_t elem, h;
    };
    int64_t k = 0;
    int64_t n = 0;                 // heap size
    std::vector<int64_t> hh, he;   // [<= k + 2], index 0 unused, index n + 1 = fixDown slack
    int64_t max_hash = INT64_MIN;  // Sampler.scala:392
    // element set: open addressing, linear probing, one int64 per slot; kEmpty marks a free slot
    // and the element equal to kEmpty (if present) is tracked by a flag instead
    static constexpr int64_t kEmpty = (int64_t)0x8000000000000001ull;
    std::vector<int64_t> slots;
    uint64_t mask = 0;
    bool has_empty = false;
    bool set_ok = true;  // false after sample_run_unique: the set is rebuilt from the heap on demand

    int64_t size() const { return n; }
    static uint64_t mix(int64_t v) {
        uint64_t z = (uint64_t)v * 0x9E3779B97F4A7C15ull;
        return z ^ (z >> 29);
    }
    void set_reserve(int64_t want) {
        uint64_t cap = 16;
        while (cap < 2 * (uint64_t)want + 2) cap <<= 1;
        if (cap <= mask + 1 && !slots.empty()) return;
        std::vector<int64_t> old;
        old.swap(slots);
        slots.assign(cap, kEmpty);
        mask = cap - 1;
        for (const int64_t x : old)
            if (x != kEmpty) set_add(x);
    }
    void prefetch(int64_t v) const { __builtin_prefetch(&slots[mix(v) & mask]); }
    void rebuild_set() {
        slots.clear();
        mask = 0;
        has_empty = false;
        set_reserve(std::max<int64_t>(n, std::min<int64_t>(k, 1 << 16)));
        for (int64_t i = 1; i <= n; ++i) set_add(he[(size_t)i]);
        set_ok = true;
    }
    bool contains(int64_t v) const {
        if (v == kEmpty) return has_empty;
        for (uint64_t q = mix(v) & mask;; q = (q + 1) & mask) {
            const int64_t s = slots[q];
            if (s == v) return true;
            if (s == kEmpty) return false;
        }
    }
    void set_add(int64_t v) {
        if (v == kEmpty) {
            has_empty = true;
            return;
        }
        uint64_t q = mix(v) & mask;
        while (slots[q] != kEmpty) q = (q + 1) & mask;
        slots[q] = v;
    }
    void set_remove(int64_t v) {
        if (v == kEmpty) {
            has_empty = false;
            return;
        }
        uint64_t p = mix(v) & mask;
        while (slots[p] != v) p = (p + 1) & mask;
        slots[p] = kEmpty;
        for (uint64_t q = (p + 1) & mask; slots[q] != kEmpty; q = (q + 1) & mask) {  // backward-shift deletion
            const uint64_t home = mix(slots[q]) & mask;
            const bool move = p <= q ? (home <= p || home > q) : (home <= p && home > q);
            if (move) {
                slots[p] = slots[q];
                slots[q] = kEmpty;
                p = q;
            }
        }
    }
    void pq_add(int64_t elem, int64_t h) {  // addOne + fixUp: parent < child -> swap
        if (n + 2 >= (int64_t)hh.size()) {  // grown on demand (doubling, at most k + 2)
            const size_t cap = (size_t)std::min<int64_t>(k + 2, std::max<int64_t>(1024, 2 * (n + 2)));
            hh.resize(cap, INT64_MIN);
            he.resize(cap, 0);
        }
        int64_t* H = hh.data();
        int64_t* E = he.data();
        int64_t m = ++n;
        while (m > 1 && H[m >> 1] < h) {
            H[m] = H[m >> 1];
            E[m] = E[m >> 1];
            m >>= 1;
        }
        H[m] = h;
        E[m] = elem;
    }
    int64_t pq_dequeue() {  // returns the removed element
        int64_t* H = hh.data();
        int64_t* E = he.data();
        const int64_t res = E[1];
        const int64_t h = H[n], e = E[n];
        const int64_t nn = --n;
        if (nn == 0) return res;
        H[nn + 1] = h;  // slack: a right child past the end compares equal to the sinking entry
        const int64_t last = (int64_t)hh.size() - 1;
        int64_t kk = 1;
        while (nn >= 2 * kk) {  // fixDown: larger child (left on ties); stop when parent >= child
            int64_t j = 2 * kk;
            __builtin_prefetch(H + std::min(4 * j, last));  // the grandchildren's line
            __builtin_prefetch(H + std::min(8 * j, last));  // and the two below it
            __builtin_prefetch(H + std::min(8 * j + 8, last));
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
    // RandomValues.sample for one element whose scrambled hash is h (Sampler.scala:394-409)
    void sample(int64_t elem, int64_t h) {
        if (!set_ok) rebuild_set();
        if (n < k) {
            if (!contains(elem)) {
                if (n + 1 > (int64_t)(mask + 1) / 2 - 1) set_reserve(2 * n + 2);
                pq_add(elem, h);
                set_add(elem);
                if (h > max_hash) max_hash = h;
            }
        } else if (h < max_hash && !contains(elem)) {
            set_remove(pq_dequeue());
            pq_add(elem, h);
            set_add(elem);
            max_hash = hh[1];
            prefetch(he[1]);  // the next replacement removes the new root from the set
        }
    }
    // sample() over a run in arrival order: elem(t), hash(t) for t in [0, c).  Once the heap is
    // full, the set probe of the next few survivors of `h < maxHash` is prefetched (maxHash only
    // falls, so a later rejection merely wastes a prefetch).
    template <typename ElemAt, typename HashAt>
    void sample_run(int64_t c, ElemAt elem, HashAt hash) {
        if (!set_ok) rebuild_set();
        constexpr int64_t kAhead = 8;
        int64_t t = 0;
        for (; t < c && n < k; ++t) sample(elem(t), hash(t));
        for (int64_t p = t; p < std::min(c, t + kAhead); ++p)
            if (hash(p) < max_hash) prefetch(elem(p));
        for (; t < c; ++t) {
            const int64_t p = t + kAhead;
            if (p < c && hash(p) < max_hash) prefetch(elem(p));
            const int64_t h = hash(t);
            if (h < max_hash) sample(elem(t), h);
        }
    }
    // The same run when first[t] != 0 exactly for the entries whose key neither occurs earlier in
    // the run nor is a member when it starts (the others cannot be admitted, see the header)
    template <typename ElemAt, typename HashAt>
    void sample_run_unique(int64_t c, const uint8_t* first, ElemAt elem, HashAt hash) {
        set_ok = false;
        int64_t t = 0;
        for (; t < c && n < k; ++t)
            if (first[t]) {
                const int64_t h = hash(t);
                pq_add(elem(t), h);
                if (h > max_hash) max_hash = h;
            }
        for (; t < c; ++t) {
            const int64_t h = hash(t);
            if (h < max_hash && first[t]) {
                pq_dequeue();
                pq_add(elem(t), h);
                max_hash = hh[1];
            }
        }
    }
    void reset(int64_t kk) {
        k = kk;
        n = 0;
        hh.assign((size_t)std::min<int64_t>(kk + 2, 1 << 17), INT64_MIN);
        he.assign(hh.size(), 0);
        max_hash = INT64_MIN;
        slots.clear();
        mask = 0;
        has_empty = false;
        set_ok = true;
        set_reserve(std::min<int64_t>(kk, 1 << 16));
    }
};

// The same replica for fixed-width byte keys (B = java.util.UUID or a case class of primitives,
// `words` 64-bit words each): the heap orders (hash, member slot) with the scala PriorityQueue tie
// behaviour above; members live in a slot pool of rows; the element set probes by the scrambled hash
// (equal keys have equal hashes) and compares the rows -- `elements.contains(elem)` is B.equals,
// which for these types is equality of the bytes.
struct HostValuesWide {
    int64_t k = 0, words = 0;
    int64_t n = 0;                 // heap size
    std::vector<int64_t> hh;       // heap hashes, 1-indexed, index n + 1 = fixDown slack
    std::vector<int32_t> hs;       // heap member slots
    std::vector<uint64_t> rows;    // slot s: rows[s * words ..)
    std::vector<int64_t> slot_h;   // hash of the member in slot s
    std::vector<int32_t> free_slots;
    std::vector<int32_t> tab;      // open addressing over member slots, -1 = free
    uint64_t mask = 0;
    int64_t max_hash = INT64_MIN;  // Sampler.scala:392

    static uint64_t mix(int64_t h) {
        uint64_t z = (uint64_t)h * 0x9E3779B97F4A7C15ull;
        return z ^ (z >> 31);
    }
    const uint64_t* row(int32_t s) const { return rows.data() + (size_t)s * words; }
    bool same(int32_t s, int64_t h, const uint64_t* r) const {
        if (slot_h[(size_t)s] != h) return false;
        const uint64_t* a = row(s);
        for (int64_t w = 0; w < words; ++w)
            if (a[w] != r[w]) return false;
        return true;
    }
    void rehash(uint64_t cap) {
        tab.assign(cap, -1);
        mask = cap - 1;
        for (int64_t i = 1; i <= n; ++i) tab_add(hs[(size_t)i]);
    }
    void tab_add(int32_t s) {
        uint64_t q = mix(slot_h[(size_t)s]) & mask;
        while (tab[q] >= 0) q = (q + 1) & mask;
        tab[q] = s;
    }
    bool contains(int64_t h, const uint64_t* r) const {
        for (uint64_t q = mix(h) & mask;; q = (q + 1) & mask) {
            const int32_t s = tab[q];
            if (s < 0) return false;
            if (same(s, h, r)) return true;
        }
    }
    void tab_remove(int32_t s) {
        uint64_t p = mix(slot_h[(size_t)s]) & mask;
        while (tab[p] != s) p = (p + 1) & mask;
        tab[p] = -1;
        for (uint64_t q = (p + 1) & mask; tab[q] >= 0; q = (q + 1) & mask) {  // backward-shift deletion
            const uint64_t home = mix(slot_h[(size_t)tab[q]]) & mask;
            const bool move = p <= q ? (home <= p || home > q) : (home <= p && home > q);
            if (move) {
                tab[p] = tab[q];
                tab[q] = -1;
                p = q;
            }
        }
    }
    int32_t alloc(int64_t h, const uint64_t* r) {
        int32_t s;
        if (!free_slots.empty()) {
            s = free_slots.back();
            free_slots.pop_back();
        } else {
            s = (int32_t)slot_h.size();
            slot_h.push_back(0);
            rows.resize(rows.size() + (size_t)words);
        }
        slot_h[(size_t)s] = h;
        std::copy(r, r + words, rows.begin() + (std::ptrdiff_t)((size_t)s * words));
        return s;
    }
    void pq_add(int32_t s, int64_t h) {  // addOne + fixUp: parent < child -> swap
        if (n + 2 >= (int64_t)hh.size()) {
            const size_t cap = (size_t)std::min<int64_t>(k + 2, std::max<int64_t>(1024, 2 * (n + 2)));
            hh.resize(cap, INT64_MIN);
            hs.resize(cap, -1);
        }
        int64_t m = ++n;
        while (m > 1 && hh[(size_t)(m >> 1)] < h) {
            hh[(size_t)m] = hh[(size_t)(m >> 1)];
            hs[(size_t)m] = hs[(size_t)(m >> 1)];
            m >>= 1;
        }
        hh[(size_t)m] = h;
        hs[(size_t)m] = s;
    }
    int32_t pq_dequeue() {  // dequeue + fixDown: larger child (left on ties), stop when parent >= child
        // (HostValues::pq_dequeue's form: the sinking hash in the slack slot past the end makes the
        // child choice one branch-free compare; the grandchildren's lines are prefetched)
        int64_t* H = hh.data();
        int32_t* S = hs.data();
        const int32_t res = S[1];
        const int64_t h = H[n];
        const int32_t e = S[n];
        const int64_t nn = --n;
        if (nn == 0) return res;
        H[nn + 1] = h;
        const int64_t last = (int64_t)hh.size() - 1;
        int64_t kk = 1;
        while (nn >= 2 * kk) {
            int64_t j = 2 * kk;
            __builtin_prefetch(H + std::min(4 * j, last));
            __builtin_prefetch(H + std::min(8 * j, last));
            __builtin_prefetch(H + std::min(8 * j + 8, last));
            j += H[j] < H[j + 1];
            if (h >= H[j]) break;
            H[kk] = H[j];
            S[kk] = S[j];
            kk = j;
        }
        H[kk] = h;
        S[kk] = e;
        return res;
    }
    void insert(int64_t h, const uint64_t* r) {
        if ((uint64_t)(n + 1) * 2 + 2 > mask + 1) rehash(std::max<uint64_t>(16, (mask + 1) * 2));
        const int32_t s = alloc(h, r);
        pq_add(s, h);
        tab_add(s);
    }
    // RandomValues.sample for one element with scrambled hash h and row r (Sampler.scala:394-409)
    void sample(int64_t h, const uint64_t* r) {
        if (n < k) {
            if (!contains(h, r)) {
                insert(h, r);
                if (h > max_hash) max_hash = h;
            }
        } else if (h < max_hash && !contains(h, r)) {
            const int32_t old = pq_dequeue();  // elements -= samples.dequeue()._1
            tab_remove(old);
            free_slots.push_back(old);
            insert(h, r);
            max_hash = hh[1];
        }
    }
    // RandomValues.sample for an element known to be the FIRST occurrence of its key since the
    // replica's state (flagged on the device): no member carries its key, so `contains` is false and
    // the element set is not consulted; a later repeat of it could never be admitted (the heap's
    // maximum never rises), so repeats are simply skipped.  The table is stale until table_rebuild().
    void sample_first(int64_t h, const uint64_t* r) {
        if (n < k) {
            pq_add(alloc(h, r), h);
            if (h > max_hash) max_hash = h;
        } else if (h < max_hash) {
            free_slots.push_back(pq_dequeue());
            pq_add(alloc(h, r), h);
            max_hash = hh[1];
        }
    }
    // sample_first for log entry `pos` of a run whose rows stay in place until adopt(): the heap holds
    // -1 - pos instead of a pool slot, so a replacement moves no row and touches no slot pool (the
    // UUID twin replay: the row copy into a recycled slot was a cache miss per replacement)
    void sample_first_at(int64_t h, int64_t pos) {
        if (n < k) {
            pq_add((int32_t)(-1 - pos), h);
            if (h > max_hash) max_hash = h;
        } else if (h < max_hash) {
            const int32_t old = pq_dequeue();
            if (old >= 0) free_slots.push_back(old);
            pq_add((int32_t)(-1 - pos), h);
            max_hash = hh[1];
        }
    }
    // the members still naming log entries take pool slots with their rows (run rows: log_rows)
    void adopt(const uint64_t* log_rows) {
        for (int64_t i = 1; i <= n; ++i) {
            const int32_t s = hs[(size_t)i];
            if (s < 0) hs[(size_t)i] = alloc(hh[(size_t)i], log_rows + (size_t)(-1 - (int64_t)s) * words);
        }
    }
    void table_rebuild() {
        uint64_t cap = 16;
        while (cap < (uint64_t)(n + 1) * 2 + 2) cap *= 2;
        rehash(cap);
    }
    // the members as (hash, row) in heap order (no sort: for the device, which orders them itself)
    void members_heap(std::vector<int64_t>& out_h, std::vector<uint64_t>& out_rows) const {
        out_h.resize((size_t)n);
        out_rows.resize((size_t)(n * words));
        for (int64_t i = 0; i < n; ++i) {
            const int32_t s = hs[(size_t)i + 1];
            out_h[(size_t)i] = hh[(size_t)i + 1];
            std::copy(row(s), row(s) + words, out_rows.begin() + (std::ptrdiff_t)(i * words));
        }
    }
    // the members as (hash, row) ascending by (hash, row words) -- the device set's order
    void members(std::vector<int64_t>& out_h, std::vector<uint64_t>& out_rows) const {
        std::vector<int32_t> ord(hs.begin() + 1, hs.begin() + 1 + n);
        std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) {
            if (slot_h[(size_t)a] != slot_h[(size_t)b]) return slot_h[(size_t)a] < slot_h[(size_t)b];
            return std::lexicographical_compare(row(a), row(a) + words, row(b), row(b) + words);
        });
        out_h.resize((size_t)n);
        out_rows.resize((size_t)(n * words));
        for (int64_t i = 0; i < n; ++i) {
            out_h[(size_t)i] = slot_h[(size_t)ord[(size_t)i]];
            std::copy(row(ord[(size_t)i]), row(ord[(size_t)i]) + words, out_rows.begin() + (std::ptrdiff_t)(i * words));
        }
    }
    void reset(int64_t kk, int64_t wwords) {
        k = kk;
        words = wwords;
        n = 0;
        hh.assign((size_t)std::min<int64_t>(kk + 2, 1 << 12), INT64_MIN);
        hs.assign(hh.size(), -1);
        rows.clear();
        slot_h.clear();
        free_slots.clear();
        max_hash = INT64_MIN;
        rehash(16);
    }
};

}  // namespace rsv
