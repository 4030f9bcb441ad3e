"""The reference's own Algorithm L (engine "java_l"): bit-identical to the reference Sampler under
the same java.util.Random seed (parity contract P1: eviction events replayed on the GPU)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def test_survey_vector_on_gpu(cuda):
    """SamplerTest.scala:117-142 setup under useConsistentRandom -> SURVEY.md 8(c) vector."""
    from reservoir_amd import Sampler

    want = GOLDEN["survey_k20"]["result"]
    s1 = Sampler(20, engine="java_l", seed=0, key_type="int")()
    for x in range(1, 3001):
        s1.sample(x)
    s2 = Sampler(20, engine="java_l", seed=0, key_type="int")()
    s2.sample_all(range(1, 1001))
    s2.sample_all(list(range(1001, 2001)))
    s2.sample_all(np.arange(2001, 3001, dtype=np.int32))
    assert s1.result().tolist() == want
    assert s2.result().tolist() == want


@pytest.mark.parametrize("case", GOLDEN["algo_l"], ids=lambda c: f"k{c['k']}_n{c['n']}_s{c['seed']}")
def test_golden_algo_l(cuda, case):
    from reservoir_amd import Sampler

    s = Sampler(case["k"], engine="java_l", seed=case["seed"])()
    s.sample_all(np.arange(1, case["n"] + 1, dtype=np.int64))
    assert s.result().tolist() == case["result"]


@pytest.mark.parametrize("k", [1, 3, 5, 64, 100, 1000, 1024, 65_537])
def test_random_keys_vs_oracle(cuda, oracle, k):
    import torch

    from reservoir_amd import Sampler

    n = 400_000
    keys = oracle.splitmix_keys(k, n)
    ref = oracle.AlgoL(k, 1234 + k)
    ref.sample_all(keys)
    s = Sampler(k, engine="java_l", seed=1234 + k)()
    kd = torch.from_numpy(keys).to(cuda)
    s.sample_all(kd[:12345])
    s.sample_all(kd[12345:])
    assert np.array_equal(s.result(), ref.result())


def test_replay_events_entry_point(cuda, oracle):
    """rsv_replay_events applies an externally generated event list (K1')."""
    import torch

    from reservoir_amd import batch

    n, k = 100_000, 77
    keys = oracle.splitmix_keys(3, n)
    ref = oracle.AlgoL(k, 5)
    ref.sample_all(keys)
    pos, slot = ref.events()
    res = batch.replay_events(torch.from_numpy(keys).to(cuda), 0, torch.from_numpy(pos),
                              torch.from_numpy(slot), k)
    assert np.array_equal(res.cpu().numpy(), ref.result())
