// C++ mirror test (reservoir/Sampler.hpp over the C ABI): the reference's SamplerTest cases that
// need no statistics, plus bit-exact checks against values the oracle wrote to argv[1].
// Built and run by tests/test_gpu_cpp.py.
#include <algorithm>
#include <cstdio>
#include <functional>
#include <fstream>
#include <numeric>
#include <string>
#include <vector>

#include "reservoir/Sampler.hpp"

using reservoir::Sampler;

static int failures = 0;
#define EXPECT(c)                                                        \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                  \
        }                                                                \
    } while (0)

template <class F, class E>
static bool throws(F f) {
    try {
        f();
    } catch (const E&) {
        return true;
    } catch (...) {
        return false;
    }
    return false;
}

int main(int argc, char** argv) {
    auto id = [](const int& x) { return (int32_t)x; };
    // SamplerTest.scala:73-79
    EXPECT((throws<std::function<void()>, reservoir::IllegalArgumentException>([&] { Sampler<int, int32_t>::apply(-1, false, false, id); })));
    EXPECT((throws<std::function<void()>, reservoir::IllegalArgumentException>([&] { Sampler<int, int32_t>::apply(2147483647, false, false, id); })));
    EXPECT((throws<std::function<void()>, reservoir::NullPointerException>([&] { Sampler<int, int32_t>::apply(5, false, false, nullptr); })));
    // :81-91
    {
        auto s = Sampler<int, int32_t>::apply(5, false, false, id);
        std::vector<int> xs(5);
        std::iota(xs.begin(), xs.end(), 1);
        s->sampleAll(xs);
        auto r = s->result();
        std::sort(r.begin(), r.end());
        EXPECT((r == std::vector<int32_t>{1, 2, 3, 4, 5}));
        EXPECT(!s->isOpen());
        EXPECT((throws<std::function<void()>, reservoir::IllegalStateException>([&] { s->sample(1); })));
    }
    {
        auto s = Sampler<int, int32_t>::apply(1, false, false, id);
        EXPECT(s->result().empty());
    }
    // :320-338 duplicates
    {
        auto s = Sampler<int, int32_t>::apply(10, false, false, id);
        auto d = Sampler<int, int32_t>::distinct(10, false, id);
        for (int i = 0; i < 10; ++i) {
            s->sample(1);
            d->sample(1);
        }
        EXPECT((s->result() == std::vector<int32_t>(10, 1)));
        EXPECT((d->result() == std::vector<int32_t>{1}));
    }
    // reusable: :273-290
    {
        auto s = Sampler<int, int32_t>::apply(64, false, true, id);
        s->result();
        s->sample(1);
        EXPECT((s->result() == std::vector<int32_t>{1}));
        EXPECT(s->isOpen());
    }
    // survey vector (SamplerTest.scala:117-142 setup, engine java_l) and an oracle-written case
    {
        reservoir::Options o;
        o.engine = reservoir::Engine::JavaL;
        o.has_seed = true;
        o.seed = 0;
        auto s = Sampler<int, int32_t>::apply(20, false, false, id, o);
        for (int x = 1; x <= 3000; ++x) s->sample(x);
        EXPECT((s->result() == std::vector<int32_t>{1335, 1173, 2365, 2555, 705, 392, 612, 786, 1639, 2529, 2575,
                                                    2058, 176, 780, 339, 607, 1147, 1511, 1218, 222}));
    }
    if (argc > 1) {  // lines: k seed stream n / expected reservoir (Algorithm R over keys 0..n-1)
        std::ifstream in(argv[1]);
        int k;
        uint64_t seed, stream;
        long n;
        while (in >> k >> seed >> stream >> n) {
            std::vector<int64_t> want((size_t)std::min<long>(n, k));
            for (auto& v : want) in >> v;
            reservoir::Options o;
            o.has_seed = true;
            o.seed = seed;
            o.stream_id = stream;
            auto s = Sampler<long, int64_t>::apply(k, false, false, [](const long& x) { return (int64_t)x; }, o);
            std::vector<long> xs((size_t)n);
            std::iota(xs.begin(), xs.end(), 0L);
            s->sampleAll(xs);
            EXPECT(s->result() == want);
        }
    }
    std::printf("%s (%d failures)\n", failures ? "FAIL" : "OK", failures);
    return failures ? 1 : 0;
}
