"""The synthetic config inputs (tools/workloads.py) have the shape SURVEY.md 8(d) prescribes (CPU)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import workloads as W  # noqa: E402


def test_splitmix_matches_oracle(oracle):
    out = torch.empty(1000, dtype=torch.int64)
    W.splitmix_fill(out, 0x5EED0000)
    assert np.array_equal(out.numpy(), oracle.splitmix_keys(0x5EED0000, 1000))


def test_feistel_is_a_permutation():
    for n in (1, 2, 3, 1000, 65_537, 1 << 20):
        p = W.feistel_perm(n, 7, "cpu").numpy()
        assert np.array_equal(np.sort(p), np.arange(n))
    assert not np.array_equal(W.feistel_perm(1000, 7, "cpu").numpy(), np.arange(1000))


def test_c4_data_duplicates():
    n = 200_000
    x = W.c4_data(n, "cpu").numpy()
    assert np.unique(x).size == int(round(n * 0.7))
    assert not np.array_equal(x[:10], np.sort(x[:10]))


def test_hash_twins_fold_hashcode(oracle):
    keys = torch.from_numpy(oracle.splitmix_keys(5, 10_000))
    tw = W.hash_twins(keys, 12).numpy()
    hc = np.array([oracle.lib().or_java_long_hashcode(int(v)) for v in tw[:2000]])
    assert hc.min() >= 0 and hc.max() < 4096
    assert np.unique(tw).size == tw.size


@pytest.mark.parametrize("n", [1000, 100_003, 2**16, 2**16 + 1])
def test_c4_slice_equals_scatter_construction(n):
    """c4_slice (inverse Feistel, any piece on its own) == the defining scatter construction, and
    the pieces of an 8-way split concatenate to the whole sequence."""
    want = W.c4_data_scatter(n, "cpu", chunk=1 << 12)
    assert torch.equal(W.c4_data(n, "cpu", chunk=1 << 12), want)
    bounds = [n * r // 8 for r in range(9)]
    pieces = [W.c4_slice(n, a, b, "cpu", chunk=1 << 12) for a, b in zip(bounds[:-1], bounds[1:])]
    assert torch.equal(torch.cat(pieces), want)
