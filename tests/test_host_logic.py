"""Host-side logic on CPU: the Sampler mirror's validation and the akka Sample-operator semantics
(SampleImpl.scala:27-57), driven with an oracle-backed stand-in sampler (no GPU here)."""
import os

import numpy as np
import pytest

import reservoir_amd
from reservoir_amd import (AbruptStageTerminationException, IllegalArgumentException,
                           NullPointerException, Sample, Sampler)
from reservoir_amd import stream as S


def test_factory_validation_matches_reference():
    # Sampler.scala:79-83, :90-95; SamplerTest.scala:73-79
    with pytest.raises(IllegalArgumentException):
        Sampler(-1)(lambda x: x)
    with pytest.raises(IllegalArgumentException):
        Sampler(2**31 - 1)(lambda x: x)
    with pytest.raises(NullPointerException):
        Sampler(5)(None)
    with pytest.raises(NullPointerException):
        Sampler.distinct(5)(lambda x: x, None)
    with pytest.raises(IllegalArgumentException):
        Sampler.distinct(0)(lambda x: x)
    # the akka factories validate eagerly too (Sample.scala:52, :89)
    with pytest.raises(IllegalArgumentException):
        Sample(-1)(lambda x: x)
    with pytest.raises(IllegalArgumentException):
        Sample.distinct(2**31 - 1)(lambda x: x)
    with pytest.raises(NullPointerException):
        Sample.distinct(3)(lambda x: x, None)


class FakeSampler:
    """CPU stand-in with the Sampler protocol (oracle Algorithm L underneath)."""

    def __init__(self, k):
        from oracle import oracle as O

        self.s = O.AlgoL(k, 1)
        self.is_open = True
        self.seen = []

    def sample(self, x):
        self.seen.append(x)
        self.s.sample(x)

    def result(self):
        self.is_open = False
        return self.s.result()


@pytest.fixture
def fake(monkeypatch):
    made = []

    def factory(k, pre_allocate=False, **ext):
        def make(map_fn):
            f = FakeSampler(k)
            made.append(f)
            return f
        return make

    monkeypatch.setattr(S, "Sampler", factory)
    return made


def test_flow_passes_elements_and_completes(fake):
    out, fut = Sample(5)(lambda x: x).run(range(1, 21))
    assert not fut.done()
    assert list(out) == list(range(1, 21))  # pass-through (SampleImpl.scala:27-31)
    assert fut.done() and len(fut.result()) == 5  # onUpstreamFinish (:38-41)
    assert fake[0].seen == list(range(1, 21))


def test_flow_is_reusable_and_lazy(fake):
    flow = Sample(3)(lambda x: x)
    assert fake == []  # by-name sampler: built when run (Sample.scala:23-24)
    for _ in range(3):
        out, fut = flow.run(range(10))
        list(out)
        assert len(fut.result()) == 3
    assert len(fake) == 3


def test_flow_upstream_failure_fails_future(fake):
    def source():
        yield 1
        yield 2
        raise ValueError("boom")

    out, fut = Sample(5)(lambda x: x).run(source())
    with pytest.raises(ValueError):
        list(out)
    with pytest.raises(ValueError):
        fut.result()  # onUpstreamFailure (:43-46)


def test_flow_downstream_cancel_completes_with_partial_sample(fake):
    out, fut = Sample(4)(lambda x: x).run(range(100))
    got = [next(out) for _ in range(10)]
    out.close()  # NonFailureCancellation (:48-54)
    assert got == list(range(10))
    assert set(fut.result().tolist()) <= set(range(10))
    assert len(fut.result()) == 4


def test_flow_empty_source(fake):
    out, fut = Sample(1)(lambda x: x).run([])
    assert list(out) == []
    assert len(fut.result()) == 0  # SampleTest.scala:72


def test_flow_downstream_failure_fails_future(fake):
    out, fut = Sample(2)(lambda x: x).run(range(10))
    next(out)
    with pytest.raises(RuntimeError):
        out.throw(RuntimeError("downstream failed"))
    with pytest.raises(RuntimeError, match="downstream failed"):
        fut.result()  # onDownstreamFinish with a failure cause (:48-54)


def test_flow_abrupt_termination(fake, monkeypatch):
    out, fut = Sample(2)(lambda x: x).run(range(10))
    next(out)
    monkeypatch.setattr(FakeSampler, "sample", lambda self, x: (_ for _ in ()).throw(OSError("device")))
    with pytest.raises(OSError):
        next(out)  # the stage fails inside onPush
    with pytest.raises(AbruptStageTerminationException):
        fut.result()  # postStop without completion (:56-57)


def test_exports():
    for name in ("Sampler", "Sample", "IllegalStateException", "ReservoirError"):
        assert hasattr(reservoir_amd, name)
    assert np.int64 is reservoir_amd.sampler._KEY["long"][1]


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N launches N ranks itself; with fewer visible GPUs it fails loudly (exit 2)
    instead of running one rank (this container has no GPU)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env={**os.environ, "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 2, r.stdout + r.stderr
    assert "--gpus 2 needs 2 visible GPUs" in r.stderr
