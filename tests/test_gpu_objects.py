"""Sampler[A, B] for any B (round 6: ObjectSampler.scala's protocol, Python key_type="object"): the
engine decides which element each slot holds from the element indices alone (rsv_sample_indexed +
rsv_commit_indexed) and the host keeps the B values -- tuples, strings, anything.  The slots must hold
exactly the elements the keyed sampler would (the oracle's last writers for philox_r; the reference's
Algorithm L for java_l, Sampler.scala:248-273), whatever mix of sample() / sampleAll(IndexedSeq) /
sampleAll(iterator); a throwing map drops its batch (rsv_abort_indexed) and leaves the sampler usable."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _expected(oracle, engine, k, n, seed=12, stream=34):
    if engine == "philox_r":
        w = oracle.algo_r_last_writers(seed, stream, k, 0, n)
        return w[w >= 0].tolist()
    ref = oracle.AlgoL(k, seed)
    ref.sample_all_iota(0, n)
    return ref.result().tolist()


@pytest.mark.parametrize("engine", ["philox_r", "java_l"])
@pytest.mark.parametrize("k,n", [(1, 1000), (100, 50), (1024, 300_000), (70_000, 200_000)])
def test_objects_every_form(cuda, oracle, engine, k, n):
    from reservoir_amd import Sampler

    seq = [("elem", i) for i in range(n)]
    s = Sampler(k, seed=12, stream_id=34, engine=engine, key_type="object")(lambda t: f"B{t[1]}")
    a, b = n // 5, n // 2
    for x in seq[:a]:                      # per element (buffered, flushed by index)
        s.sample(x)
    s.sample_all(iter(seq[a:a + 10]))      # an iterator: per element
    s.sample_all(seq[a + 10:b])            # an IndexedSeq: map on the winners only
    s.sample_all(tuple(seq[b:]))
    want = [f"B{i}" for i in _expected(oracle, engine, k, n)]
    assert s.result() == want
    assert not s.is_open


def test_objects_throwing_map_and_reusable(cuda, oracle):
    from reservoir_amd import IllegalStateException, Sampler

    k, n = 512, 400_000
    calls = []

    def boom(x):
        calls.append(x)
        if len(calls) == 3:
            raise ValueError("map threw")
        return x * 10

    s = Sampler(k, reusable=True, seed=12, stream_id=34, key_type="object")(lambda x: x * 10)
    s.sample_all(range(1000))
    first = s.result()
    assert first == [10 * i for i in _expected(oracle, "philox_r", k, 1000)]
    s._map = boom  # the next batch's map throws on its third call
    with pytest.raises(ValueError):
        s.sample_all(range(1000, n))
    assert s.result() == first  # the batch was dropped as a whole
    s._map = lambda x: x * 10
    s.sample_all(range(1000, n))
    assert s.result() == [10 * i for i in _expected(oracle, "philox_r", k, n)]
    assert s.is_open
    s.close()
    with pytest.raises(IllegalStateException):
        s.sample(1)


def test_objects_c2_scale(cuda, oracle):
    """1e9 elements as one IndexedSeq (a range of element ids): map runs on <= k of them"""
    from reservoir_amd import Sampler

    n, k = 1_000_000_000, 1024
    mapped = []
    s = Sampler(k, seed=12, stream_id=34, key_type="object")(lambda i: mapped.append(i) or ("id", i))
    s.sample_all(range(n))
    assert len(mapped) <= k
    assert s.result() == [("id", i) for i in _expected(oracle, "philox_r", k, n)]
