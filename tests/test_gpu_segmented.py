"""Segmented sampling (K2): S independent samplers per launch.  Parity with the oracle on ragged
inputs, and the reference's 5-sigma fairness/independence tests (SamplerTest.scala:156-240) run
with 1e6 independent samplers in one launch."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k", [1, 5, 64, 100, 1024, 3000, 4400, 4416, 4417, 8192, 65536])
def test_ragged_parity(cuda, oracle, k):
    """k < 512: one wave per stream (k2_segmented); from k = 512 one workgroup per stream with one
    shared table (k2_segmented_wg): in LDS up to k ~ 29.5k (u32 entries), beyond that a slice of the
    persistent global scratch (k = 65536)."""
    import torch

    from reservoir_amd import batch

    rng = np.random.default_rng(k)
    big = k > 4096
    lens = rng.integers(0, 4 * k + 5000 if big else 5000, size=60 if big else 300)
    lens[:6] = [0, 1, k - 1 if k > 1 else 0, k, k + 1, 4096]
    offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
    keys = oracle.splitmix_keys(k, int(offs[-1]))
    want, wcnt = oracle.algo_r_segmented(77, 1000, k, keys, offs)
    out, cnt = batch.sample_segmented(torch.from_numpy(keys).to(cuda), torch.from_numpy(offs).to(cuda), k,
                                      seed=77, stream_base=1000)
    assert np.array_equal(cnt.cpu().numpy(), wcnt)
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("k", [1, 2, 3, 17, 63, 64])
def test_two_deep_gather_stream_counts(cuda, oracle, k):
    """k <= 64 gathers each stream's winners two streams later (rsv_k2.h, slot u waited on with an
    explicit vmcnt(2)): odd and even numbers of streams per wave, and the launch's last streams
    (a wave's final one or two slots drained after its loop), vs the oracle."""
    import torch

    from reservoir_amd import batch

    for S in (1, 2, 3, 5, 4096 * 4 + 1, 4096 * 4 * 3 + 7, 100_003):
        rng = np.random.default_rng(S * 131 + k)
        lens = rng.integers(0, 300, size=S)
        offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
        keys = oracle.splitmix_keys(S + k, int(offs[-1]))
        want, wcnt = oracle.algo_r_segmented(5, 3, k, keys, offs)
        out, cnt = batch.sample_segmented(torch.from_numpy(keys).to(cuda), torch.from_numpy(offs).to(cuda), k,
                                          seed=5, stream_base=3)
        assert np.array_equal(cnt.cpu().numpy(), wcnt), S
        assert np.array_equal(out.cpu().numpy(), want), S


_FIFO_CASE = """
import sys
import numpy as np
import torch
sys.path.insert(0, {root!r})
from oracle import oracle
from reservoir_amd import batch
cuda = torch.device("cuda", 0)
for k in (64, 256, 1000):
    rng = np.random.default_rng(500 + k)
    lens = rng.integers(0, 20_000, size=200)
    lens[:4] = [k, k + 1, 4096, 19_999]
    offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
    keys = oracle.splitmix_keys(11 * k, int(offs[-1]))
    want, wcnt = oracle.algo_r_segmented(31, 77, k, keys, offs)
    out, cnt = batch.sample_segmented(torch.from_numpy(keys).to(cuda), torch.from_numpy(offs).to(cuda), k,
                                      seed=31, stream_base=77)
    assert np.array_equal(cnt.cpu().numpy(), wcnt), k
    assert np.array_equal(out.cpu().numpy(), want), k
print("fifo overflow ok")
"""


def test_fifo_overflow_rounds(cuda, oracle):
    """An iteration with more candidates than the FIFO takes (RSV_K2_FIFO_CAP lowers the bulk-append
    limit to 128; at k = 256 an iteration past the dense head holds ~177) goes through the ballot-
    round path of rsv_k2.h: same reservoirs as the oracle, k = 64, 256, 1000.  The engine reads the
    variable once per process, so the cases run in a child process that sets it."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RSV_K2_FIFO_CAP="128")
    r = subprocess.run([sys.executable, "-c", _FIFO_CASE.format(root=root)], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "fifo overflow ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("k", [2, 7, 64])
def test_long_streams_sparse_region(cuda, oracle, k):
    """Streams far longer than 256k: the dense head and the sparse tail (zero level-0 bytes only)."""
    import torch

    from reservoir_amd import batch

    rng = np.random.default_rng(100 + k)
    lens = np.r_[rng.integers(0, 300_000, size=12), 256 * k - 1, 256 * k, 256 * k + 17, 1_000_003]
    offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
    keys = oracle.splitmix_keys(3 * k, int(offs[-1]))
    want, wcnt = oracle.algo_r_segmented(5, 2**40 + 3, k, keys, offs)
    out, cnt = batch.sample_segmented(torch.from_numpy(keys).to(cuda), torch.from_numpy(offs).to(cuda), k,
                                      seed=5, stream_base=2**40 + 3)
    assert np.array_equal(cnt.cpu().numpy(), wcnt)
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("k", [64, 1000, 8192])
def test_streams_past_2pow27(cuda, oracle, k):
    """Streams of >= 2^27 keys take K2's 64-bit path (u64 LDS winner table, full Philox counter
    words, 64-bit index rebuild in resolve_round).  keys = arange, so each output key is its global
    index: segment s must hold offset_s + the oracle's last writer of every slot."""
    import torch

    from reservoir_amd import batch

    lens = [(1 << 27) + 12_345, max(1000, k + 808), (1 << 27) + 1]
    offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
    keys = torch.arange(int(offs[-1]), dtype=torch.int64, device=cuda)
    out, cnt = batch.sample_segmented(keys, torch.from_numpy(offs).to(cuda), k, seed=41, stream_base=9)
    out = out.cpu().numpy().reshape(len(lens), k)
    assert cnt.cpu().numpy().tolist() == [k] * len(lens)
    for s, n in enumerate(lens):
        win = oracle.algo_r_last_writers(41, 9 + s, k, 0, n)
        assert (win >= 0).all()
        assert np.array_equal(out[s], offs[s] + win), s
    del keys
    torch.cuda.empty_cache()


def test_int32_keys(cuda, oracle):
    import torch

    from reservoir_amd import batch

    offs = np.arange(0, 4096 * 50 + 1, 4096, dtype=np.int64)
    keys = (oracle.splitmix_keys(1, int(offs[-1])) >> 33).astype(np.int32)
    want, _ = oracle.algo_r_segmented(3, 0, 64, keys.astype(np.int64), offs)
    out, _ = batch.sample_segmented(torch.from_numpy(keys).to(cuda), torch.from_numpy(offs).to(cuda), 64, seed=3)
    assert np.array_equal(out.cpu().numpy().astype(np.int64), want)


def test_segment_equals_single_sampler(cuda, oracle):
    """stream s of a segmented launch == a single sampler with stream_id = stream_base + s."""
    import torch

    from reservoir_amd import Sampler, batch

    offs = np.array([0, 10_000, 10_500, 30_000], dtype=np.int64)
    keys = oracle.splitmix_keys(2, 30_000)
    kd = torch.from_numpy(keys).to(cuda)
    out, _ = batch.sample_segmented(kd, torch.from_numpy(offs).to(cuda), 128, seed=11, stream_base=40)
    for s in range(3):
        sm = Sampler(128, seed=11, stream_id=40 + s)()
        sm.sample_all(kd[offs[s]:offs[s + 1]])
        r = sm.result()
        assert np.array_equal(out[s, : r.size].cpu().numpy(), r)


def _million_trials(cuda, torch, batch, seed):
    trials, c = 1_000_000, 10
    elements = torch.arange(1, c + 1, dtype=torch.int64, device=cuda).repeat(trials)
    offs = torch.arange(0, trials * c + 1, c, dtype=torch.int64, device=cuda)
    out, cnt = batch.sample_segmented(elements, offs, c // 2, seed=seed)
    assert int(cnt.min()) == c // 2
    return out  # [trials, 5] sampled elements


def test_fairness_five_sigma_1e6(cuda):
    """SamplerTest.scala:156-176 with the reference's n = 1e6."""
    import torch

    from reservoir_amd import batch

    out = _million_trials(cuda, torch, batch, seed=2024)
    counts = torch.bincount(out.flatten(), minlength=11)[1:].cpu().numpy()
    sd = math.sqrt(1_000_000 / 4.0)
    assert np.all(np.abs(counts - 500_000) < math.ceil(5 * sd)), counts
    # no element twice in one sample (sampling without replacement)
    srt = torch.sort(out, dim=1).values
    assert bool((srt[:, 1:] != srt[:, :-1]).all())


def test_pairwise_independence_five_sigma_1e6(cuda):
    """SamplerTest.scala:198-232: pairs with the same inclusion status, within 5 sigma."""
    import torch

    from reservoir_amd import batch

    n, c = 1_000_000, 10
    out = _million_trials(cuda, torch, batch, seed=77)
    member = torch.zeros((n, c + 1), dtype=torch.bool, device=cuda)
    member.scatter_(1, out, True)
    member = member[:, 1:].to(torch.float32)
    same = member.T @ member + (1 - member).T @ (1 - member)  # [c, c] counts of equal status
    p = ((c / 2.0) - 1) / (c - 1)
    mean = round(n * p)
    sd = math.sqrt(n * p * (1 - p))
    s = same.cpu().numpy()
    off = s[~np.eye(c, dtype=bool)]
    assert np.all(np.abs(off - mean) < math.ceil(5 * sd)), off


def test_slot_chi_square(cuda):
    """Chi-square slot-inclusion uniformity (north star) at k = 64 over 4096-element streams."""
    import torch

    from reservoir_amd import batch

    S, L, k = 20_000, 4096, 64
    keys = torch.arange(L, dtype=torch.int64, device=cuda).repeat(S)  # key = index in stream
    offs = torch.arange(0, S * L + 1, L, dtype=torch.int64, device=cuda)
    out, _ = batch.sample_segmented(keys, offs, k, seed=99)
    # inclusion count of each index in 64 bins of 64 consecutive indices: uniform k/L each
    bins = torch.bincount(out.flatten() // 64, minlength=64).to(torch.float64).cpu().numpy()
    exp = S * k / 64
    chi2 = ((bins - exp) ** 2 / exp).sum()
    # sampling without replacement lowers the variance; dof 63: p(chi2 > 120) < 1e-5
    assert chi2 < 120, chi2


def test_wg_global_scratch_reuse(cuda, oracle):
    """k = 40000: the workgroup form's table lives in the per-device global scratch, zeroed once and
    left zero by every launch.  Back-to-back launches on one stream, then on a second stream while the
    first may still run (a private zeroed block), all equal the oracle."""
    import torch

    from reservoir_amd import batch

    k = 40_000
    rng = np.random.default_rng(9)
    lens = rng.integers(0, 3 * k, size=40)
    lens[:3] = [0, k, 2 * k + 7]
    offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
    keys = oracle.splitmix_keys(5, int(offs[-1]))
    want, wcnt = oracle.algo_r_segmented(3, 9, k, keys, offs)
    kd, od = torch.from_numpy(keys).to(cuda), torch.from_numpy(offs).to(cuda)
    outs = [batch.sample_segmented(kd, od, k, seed=3, stream_base=9) for _ in range(2)]
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        outs.append(batch.sample_segmented(kd, od, k, seed=3, stream_base=9))
    torch.cuda.synchronize()
    for out, cnt in outs:
        assert np.array_equal(cnt.cpu().numpy(), wcnt)
        assert np.array_equal(out.cpu().numpy(), want)
