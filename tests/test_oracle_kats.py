"""Pin the CPU oracle: third-party known answers and the committed golden vectors (CPU only)."""
import json
import os

import numpy as np
import pytest

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


# ---- java.util.Random: widely published JDK values ----------------------------------------
def test_java_random_known_answers(oracle):
    assert oracle.JavaRandom(0).next_int() == -1155484576
    assert oracle.JavaRandom(42).next_int() == -1170105035
    r = oracle.JavaRandom(0)
    assert (r.next_long(), r.next_long()) == (-4962768465676381896, 4437113781045784766)
    assert oracle.JavaRandom(0).next_double() == 0.730967787376657


def test_java_random_next_int_bound_paths(oracle):
    # power-of-two fast path: (bound * next(31)) >> 31, i.e. the top bits of next(31)
    r1, r2 = oracle.JavaRandom(5), oracle.JavaRandom(5)
    for _ in range(1000):
        v = r1.next_int(64)
        raw = r2.next_int(2**30)  # also power of two: top 30 of next(31)
        assert v == raw >> 24
    # rejection path: values in range, deterministic
    r = oracle.JavaRandom(7)
    vals = [r.next_int(100) for _ in range(10_000)]
    assert min(vals) >= 0 and max(vals) < 100
    r = oracle.JavaRandom(7)
    assert vals == [r.next_int(100) for _ in range(10_000)]


# ---- Philox4x32-10: Random123 known-answer vectors ------------------------------------------
@pytest.mark.parametrize(
    "ctr,key,want",
    [
        ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
        ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
        ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
         [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
    ],
)
def test_philox_random123_kat(oracle, ctr, key, want):
    assert oracle.philox4x32_10(ctr, key) == want


# ---- scala byteswap64 ---------------------------------------------------------------------
def test_byteswap64_is_a_bijection_sample(oracle):
    xs = np.random.default_rng(1).integers(-2**63, 2**63 - 1, size=20000, dtype=np.int64)
    ys = {oracle.byteswap64(int(x)) for x in xs}
    assert len(ys) == len(set(xs.tolist()))
    assert oracle.byteswap64(0) == 0


# ---- golden vectors ------------------------------------------------------------------------
def test_survey_vector(oracle):
    """independently restated vector for the SamplerTest.scala:117-142 setup."""
    want = [1335, 1173, 2365, 2555, 705, 392, 612, 786, 1639, 2529, 2575, 2058, 176, 780, 339, 607,
            1147, 1511, 1218, 222]
    s = oracle.AlgoL(20, 0)
    for x in range(1, 3001):
        s.sample(x)
    assert s.result().tolist() == want
    pos, slot = s.events()
    assert pos.size == 88
    assert list(zip(pos[:8].tolist(), slot[:8].tolist())) == [
        (21, 15), (22, 14), (23, 15), (25, 0), (27, 12), (31, 3), (33, 2), (36, 15)]
    assert GOLDEN["survey_k20"]["result"] == want


@pytest.mark.parametrize("case", GOLDEN["algo_l"], ids=lambda c: f"k{c['k']}_n{c['n']}_s{c['seed']}")
def test_golden_algo_l(oracle, case):
    s = oracle.AlgoL(case["k"], case["seed"])
    for x in range(1, case["n"] + 1):
        s.sample(x)
    assert s.result().tolist() == case["result"]
    pos, slot = s.events()
    assert pos.size == case["n_events"]
    assert [[int(p), int(q)] for p, q in zip(pos[:16], slot[:16])] == case["events_head"]


@pytest.mark.parametrize("case", GOLDEN["draws"], ids=lambda c: f"i0_{c['i0']}")
def test_golden_draws(oracle, case):
    j = oracle.export_draws(case["seed"], case["stream"], case["i0"], case["n"])
    assert [int(x) for x in j] == case["j"]
    for t, i in enumerate(range(case["i0"], case["i0"] + case["n"])):
        assert 0 <= case["j"][t] <= i  # j_i uniform on [0, i]


@pytest.mark.parametrize("case", GOLDEN["algo_r"], ids=lambda c: f"k{c['k']}_n{c['n']}")
def test_golden_algo_r(oracle, case):
    keys = oracle.splitmix_keys(case["key_base"], case["n"])
    res, repl = oracle.algo_r(case["seed"], case["stream"], case["k"], keys)
    assert res.tolist() == case["result"] and repl == case["replacements"]


@pytest.mark.parametrize("case", GOLDEN["distinct"], ids=lambda c: f"k{c['k']}_h{c['hash_kind']}")
def test_golden_distinct(oracle, case):
    d = oracle.Distinct(case["k"], case["seed"], case["hash_kind"])
    d.sample_all(case["values"])
    keys, hs = d.result()
    assert keys.tolist() == case["result_sorted_by_hash"]
    assert hs.tolist() == case["hashes"]
    r = oracle.JavaRandom(case["seed"])
    assert (d.r0, d.r1) == (r.next_long(), r.next_long())  # Sampler.scala:385-388
