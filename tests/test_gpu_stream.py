"""The akka Sample operator mirror (Sample.scala / SampleImpl.scala) over the GPU samplers:
SampleTest.scala's boundary cases and the element / distinct behaviours."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(flow, source):
    out, fut = flow.run(source)
    passed = list(out)
    return passed, fut.result()


@pytest.mark.parametrize("distinct", [False, True])
def test_boundaries(cuda, distinct):
    from reservoir_amd import Sample

    mk = (lambda k: Sample.distinct(k, key_type="int")(lambda x: x)) if distinct else \
         (lambda k: Sample(k, key_type="int")(lambda x: x))
    assert sorted(_run(mk(5), range(1, 6))[1].tolist()) == [1, 2, 3, 4, 5]  # SampleTest.scala:61-64
    assert sorted(_run(mk(6), range(1, 6))[1].tolist()) == [1, 2, 3, 4, 5]  # :66-69
    assert _run(mk(1), [])[1].tolist() == []  # :71-72


def test_duplicates(cuda):
    from reservoir_amd import Sample

    passed, res = _run(Sample(10, key_type="int")(lambda x: x), [1] * 10)
    assert passed == [1] * 10 and res.tolist() == [1] * 10  # SampleTest.scala:207-218
    _, res = _run(Sample.distinct(10, key_type="int")(lambda x: x), [1] * 10)
    assert res.tolist() == [1]  # :226-236


def test_sometimes_and_not_always(cuda):
    from reservoir_amd import Sample

    flow = Sample(5, key_type="int")(lambda x: x)
    got = [_run(flow, range(1, 7))[1].tolist() for _ in range(100)]
    assert any(6 in g for g in got) and any(6 not in g for g in got)  # SampleTest.scala:75-85


def test_long_stream_matches_sampler(cuda, oracle):
    """The operator's per-element path (pinned staging) equals sampleAll on the same seed."""
    from reservoir_amd import Sample, Sampler

    keys = oracle.splitmix_keys(11, 3_000_000)
    _, res = _run(Sample(1000, seed=5)(lambda x: x), (int(x) for x in keys))
    s = Sampler(1000, seed=5)()
    s.sample_all(keys)
    assert np.array_equal(res, s.result())
