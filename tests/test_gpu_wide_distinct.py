"""Sampler.distinct over fixed-width byte keys (key_type "bytesN": UUIDs, case classes of
primitives) on the HIP engine (rsv_wide.hip) vs the byte-row oracle (oracle.DistinctRows: the
reference's RandomValues, Sampler.scala:383-412, with B.equals = equal bytes).

Parity: the set equals the oracle's -- in ordered mode for ANY hash (the reference's sequential heap,
boundary bucket included: the host replay), in set mode for an injective hash.  Hashes are the
caller's precomputed Longs (RSV_HASH_PRECOMPUTED) or java.util.UUID.hashCode of 16-byte keys
(RSV_HASH_DEFAULT).  Sizes: k in {1, 100, 65536}, widths 16 / 24 / 64, device and host batches,
per-element sample(); C4's per-GPU share (5e8 keys, 30 % duplicates, k = 65536) as 16-byte UUIDs in
set mode (precomputed 64-bit hash), in ordered mode under UUID.hashCode, and as hash twins (~5 keys
per hash value) so the ordered replay runs at full size.
"""
import sys
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

M64 = (1 << 64) - 1


def _rows(ids, width):
    """width-byte key of element id (the splitmix stream of the id, little-endian words)."""
    ids = np.asarray(ids, dtype=np.uint64)
    out = np.empty((ids.size, width // 8), dtype=np.uint64)
    for w in range(width // 8):
        z = ids * np.uint64(0x9E3779B97F4A7C15) + np.uint64((w * 0x632BE59BD9B4E019 + 1) & M64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        out[:, w] = z ^ (z >> np.uint64(31))
    return out.view(np.uint8).reshape(ids.size, width)


def _stream(n, seed):
    """element ids with ~30 % repeats, in random order"""
    rng = np.random.default_rng(seed)
    d = int(n * 0.7)
    ids = np.concatenate([np.arange(d), rng.integers(0, d, n - d)])
    rng.shuffle(ids)
    return ids


def _hashes(ids, kind):
    if kind == "random":   # a 64-bit hash: injective in practice (set mode == the reference)
        return (_rows(ids, 8).view(np.int64).reshape(-1) ^ 0x5A5A).astype(np.int64)
    if kind == "collide":  # 97 hash values: the boundary bucket is oversubscribed (host replay)
        return (np.asarray(ids, dtype=np.int64) % 97) - 48
    raise ValueError(kind)


def _sorted_rows(a):
    a = np.ascontiguousarray(a)
    return sorted(bytes(r) for r in a)


def _expect(k, seed, width, rows, hashes, uuid=False):
    from oracle import oracle as O

    ref = O.DistinctRows(k, seed, width, "uuid" if uuid else "precomputed")
    ref.sample_all(rows, None if uuid else hashes)
    got, hs = ref.result()
    return _sorted_rows(got), hs


@pytest.mark.parametrize("width", [16, 24, 64])
@pytest.mark.parametrize("k", [1, 100, 65536])
@pytest.mark.parametrize("hkind,order", [("random", "set"), ("random", "auto"), ("collide", "auto")])
def test_wide_distinct_device_batches(cuda, width, k, hkind, order):
    import torch

    from reservoir_amd import Sampler

    n = 300_000 if k == 65536 else 60_000
    ids = _stream(n, k + width)
    rows = _rows(ids, width)
    hs = _hashes(ids, hkind)
    want, wh = _expect(k, 9, width, rows, hs)
    d = Sampler.distinct(k, key_type=f"bytes{width}", seed=9, order=order)(hash=lambda b: 0)
    assert d.is_ordered == (order == "auto")
    rd = torch.from_numpy(rows).to(cuda)
    hd = torch.from_numpy(hs).to(cuda)
    cut = n // 3
    d.sample_all(rd[:cut], hashes=hd[:cut])
    d.sample_all(rd[cut:], hashes=hd[cut:])
    info = d.distinct_info()
    got = d.result()
    assert got.shape == (min(k, len(want)), width)
    assert _sorted_rows(got) == want
    if hkind == "collide" and k > 1:  # the boundary bucket holds more distinct keys than kept
        assert info["tied"]


@pytest.mark.parametrize("k", [1, 100, 5000])
def test_wide_distinct_host_paths(cuda, k):
    """Host batches with a callable hash, per-element sample(), and both in one sampler."""
    from reservoir_amd import Sampler

    width = 24
    ids = _stream(30_000, k)
    rows = _rows(ids, width)

    def h(b):  # the JVM-side `hash: B => Long`: few values -> ties
        return int.from_bytes(bytes(b)[8:16], "little", signed=True) % 61

    hs = np.array([h(r.tobytes()) for r in rows], dtype=np.int64)
    want, _ = _expect(k, 4, width, rows, hs)
    d = Sampler.distinct(k, key_type=f"bytes{width}", seed=4)(hash=h)
    d.sample_all(rows[:10_000])
    for r in rows[10_000:10_500]:
        d.sample(r.tobytes())
    d.sample_all(rows[10_500:])
    assert _sorted_rows(d.result()) == want


@pytest.mark.parametrize("k", [1, 100, 65536])
def test_wide_distinct_uuid_default_hash(cuda, k):
    """16-byte keys with the default hash: java.util.UUID.hashCode on the device (ordered mode)."""
    import torch
    import workloads as W

    from reservoir_amd import Sampler

    n = 400_000
    vals = torch.from_numpy(np.random.default_rng(k).integers(-2**63, 2**63 - 1, n // 2 + 7, dtype=np.int64)).to(cuda)
    vals = torch.cat([vals, vals[: n // 2]])
    rows = W.uuid_rows(vals, twin_bits=12)  # ~50 keys per UUID.hashCode value
    d = Sampler.distinct(k, key_type="bytes16", seed=13)()
    assert d.is_ordered
    d.sample_all(rows)
    got = d.result()
    want, _ = _expect(k, 13, 16, rows.cpu().numpy(), None, uuid=True)
    assert _sorted_rows(got) == want


@pytest.mark.parametrize("k", [1, 100, 5000])
@pytest.mark.parametrize("hkind", ["random", "collide", "uuid"])
@pytest.mark.parametrize("merge", ["bucketed", "sort"])
def test_wide_sched_pass(cuda, capfd, monkeypatch, k, hkind, merge):
    """Ordered mode over one long batch takes the scheduled pass (falling per-range bounds, proved
    by wb_verify / wide_verify): equal to the oracle, to the chunk loop (RSV_WIDE_SCHED=0), and --
    with bounds made too tight (RSV_WIDE_SCHED_BETA) -- the failed proof restores the set and the log
    and the chunk loop gives the same set.  Both merges: the bucketed one (round 6: its bucket map
    follows the pass's uneven density along h) and the sort-based one (RSV_WIDE_BUCKETED=0)."""
    import torch

    from reservoir_amd import Sampler

    monkeypatch.setenv("RSV_WIDE_SCHED_DEBUG", "1")
    if merge == "sort":
        monkeypatch.setenv("RSV_WIDE_BUCKETED", "0")
    n = 400_000
    ids = _stream(n, 7 * k + len(hkind))
    rows = _rows(ids, 16)
    uuid = hkind == "uuid"
    hs = None if uuid else _hashes(ids, hkind)
    want, _ = _expect(k, 5, 16, rows, hs, uuid=uuid)
    rd = torch.from_numpy(rows).to(cuda)
    hd = None if uuid else torch.from_numpy(hs).to(cuda)

    def run(**env):
        for key, v in env.items():
            monkeypatch.setenv(key, v)
        d = Sampler.distinct(k, key_type="bytes16", seed=5)() if uuid else \
            Sampler.distinct(k, key_type="bytes16", seed=5)(hash=lambda b: 0)
        assert d.is_ordered
        d.sample_all(rd, hashes=hd)
        got = _sorted_rows(d.result())
        for key in env:
            monkeypatch.delenv(key)
        return got, capfd.readouterr().err

    got, err = run()
    assert got == want
    sched = k >= 64  # (smaller k keep the chunk loop: rsv_wide.hip kSchedMinK)
    assert ("[rsv wide sched]" in err) == sched, err
    if sched and hkind != "collide":  # (97 hash values: no k-th smallest falls below a predicted bound)
        assert "proof=ok" in err, err
        assert f"merge={merge}" in err, err  # no bucket overflowed: the map followed the density
    got0, err0 = run(RSV_WIDE_SCHED="0")
    assert got0 == want and "[rsv wide sched]" not in err0
    got1, err1 = run(RSV_WIDE_SCHED_BETA="0.02")
    assert got1 == want
    if sched:
        assert "proof=failed" in err1, err1


def test_wide_distinct_eager_replays(cuda, monkeypatch):
    """A small log limit forces the ordered log to be replayed mid-batch (several times)."""
    import torch

    from reservoir_amd import Sampler

    monkeypatch.setenv("RSV_ORDERED_LOG_LIMIT", "3000")
    ids = _stream(200_000, 3)
    rows = _rows(ids, 16)
    hs = _hashes(ids, "collide")
    want, _ = _expect(500, 2, 16, rows, hs)
    d = Sampler.distinct(500, key_type="bytes16", seed=2)(hash=lambda b: 0)
    rd, hd = torch.from_numpy(rows).to(cuda), torch.from_numpy(hs).to(cuda)
    for a in range(0, rows.shape[0], 37_000):
        d.sample_all(rd[a:a + 37_000], hashes=hd[a:a + 37_000])
    assert _sorted_rows(d.result()) == want


@pytest.mark.parametrize("first_min", ["0", "1000000000"])
@pytest.mark.parametrize("log_limit", [None, "3000"])
def test_wide_first_occurrence_replay(cuda, monkeypatch, first_min, log_limit):
    """The ordered replay through first-occurrence flags (heap only, no element set: RSV_FIRST_MIN=0)
    and through the replica's element set (RSV_FIRST_MIN huge) both equal the oracle -- colliding
    hashes, keys repeating within and across batches and logs, eager replays mid-batch."""
    import torch

    from reservoir_amd import Sampler

    monkeypatch.setenv("RSV_FIRST_MIN", first_min)
    if log_limit:
        monkeypatch.setenv("RSV_ORDERED_LOG_LIMIT", log_limit)
    ids = _stream(150_000, 21)
    ids = np.concatenate([ids, ids[:40_000]])  # whole-log repeats
    rows = _rows(ids, 24)
    hs = _hashes(ids, "collide")
    want, _ = _expect(300, 4, 24, rows, hs)
    d = Sampler.distinct(300, key_type="bytes24", seed=4)(hash=lambda b: 0)
    rd, hd = torch.from_numpy(rows).to(cuda), torch.from_numpy(hs).to(cuda)
    for a in range(0, rows.shape[0], 47_000):
        d.sample_all(rd[a:a + 47_000], hashes=hd[a:a + 47_000])
    assert _sorted_rows(d.result()) == want


def test_wide_distinct_reusable_and_long_runs(cuda):
    """A reusable sampler (result() between batches), and one hash value for every key: runs of
    equal hash far above 64 entries take the comparison-sort merge."""
    import torch

    from reservoir_amd import Sampler

    ids = _stream(50_000, 5)
    rows = _rows(ids, 32)
    hs = np.zeros(ids.size, dtype=np.int64)  # a degenerate hash
    for order in ("set", "ordered"):
        d = Sampler.distinct(300, key_type="bytes32", seed=1, reusable=True, order=order)(hash=lambda b: 0)
        rd, hd = torch.from_numpy(rows).to(cuda), torch.from_numpy(hs).to(cuda)
        for a in (0, 20_000):
            b = a + 20_000 if a == 0 else ids.size
            d.sample_all(rd[a:b], hashes=hd[a:b])
            got = d.result()
            assert got.shape[0] == 300
        if order == "ordered":  # one bucket: arrival order decides, exactly as the reference
            want, _ = _expect(300, 1, 32, rows, hs)
            assert _sorted_rows(got) == want
        else:  # set mode: the 300 smallest keys of the bucket by key words
            u = np.unique(rows.view(np.uint64).reshape(-1, 4), axis=0)[:300]
            assert _sorted_rows(got) == _sorted_rows(u.view(np.uint8))


def test_wide_distinct_export_merge(cuda):
    """Split a stream over 3 samplers (the 3 ranks of a combine), merge their packed rows on the
    device (set mode), and in ordered mode with the exact replay (merge_local)."""
    import torch

    from reservoir_amd import Sampler
    from reservoir_amd import distributed as D

    width, k = 24, 2000
    ids = _stream(150_000, 8)
    rows = _rows(ids, width)
    for hkind, order in (("random", "set"), ("collide", "ordered")):
        hs = _hashes(ids, hkind)
        want, _ = _expect(k, 6, width, rows, hs)
        rd, hd = torch.from_numpy(rows).to(cuda), torch.from_numpy(hs).to(cuda)
        cuts = [0, 40_000, 100_000, ids.size]
        shards = []
        for r in range(3):
            s = Sampler.distinct(k, key_type=f"bytes{width}", seed=6, order=order,
                                 retain_log=order == "ordered")(hash=lambda b: 0)
            s.sample_all(rd[cuts[r]:cuts[r + 1]], hashes=hd[cuts[r]:cuts[r + 1]])
            shards.append(s)
        target = Sampler.distinct(k, key_type=f"bytes{width}", seed=6, order=order)(hash=lambda b: 0)
        replayed = D.merge_local(target, shards)
        assert target.count == ids.size
        assert _sorted_rows(target.result()) == want, order
        if order == "ordered":
            assert replayed


# ------------------------------------------------------------------- C4 share as 16-byte keys
def _c4_uuid(cuda, twin_bits=None):
    import workloads as W

    vals = W.c4_data(500_000_000, cuda)
    rows = W.uuid_rows(vals, twin_bits)
    return vals, rows


@pytest.mark.timeout(600)
def test_c4_share_uuid_set_mode(cuda):
    """5e8 16-byte keys (30 % duplicates), k = 65536, a precomputed 64-bit hash, set mode."""
    import torch
    import workloads as W

    from reservoir_amd import Sampler

    vals, rows = _c4_uuid(cuda)
    hs = W.smix(vals ^ 0x5A5A)
    del vals
    d = Sampler.distinct(65536, key_type="bytes16", seed=7, order="set")(hash=lambda b: 0)
    d.sample_all(rows, hashes=hs)
    got = d.result()
    want, _ = _expect(65536, 7, 16, rows.cpu().numpy(), hs.cpu().numpy())
    assert got.shape == (65536, 16)
    assert _sorted_rows(got) == want
    del rows, hs
    torch.cuda.empty_cache()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("twin_bits", [None, 26])
def test_c4_share_uuid_ordered(cuda, twin_bits):
    """The same share under the default UUID.hashCode (ordered mode); with twin_bits = 26 about 5
    distinct keys share each hash value and the boundary bucket forces the host replay."""
    import torch

    from reservoir_amd import Sampler

    vals, rows = _c4_uuid(cuda, twin_bits)
    del vals
    d = Sampler.distinct(65536, key_type="bytes16", seed=11)()
    d.sample_all(rows)
    info = d.distinct_info()
    got = d.result()
    want, _ = _expect(65536, 11, 16, rows.cpu().numpy(), None, uuid=True)
    assert got.shape == (65536, 16)
    assert _sorted_rows(got) == want
    if twin_bits:
        assert info["tied"]
    del rows
    torch.cuda.empty_cache()


def test_wide_rejections(cuda):
    from reservoir_amd import Sampler, ReservoirError

    with pytest.raises(ReservoirError):  # no default hashCode for 24-byte keys: RSV_E_UNSUPPORTED
        Sampler.distinct(10, key_type="bytes24")()
    with pytest.raises(ReservoirError):
        Sampler.distinct(10, key_type="bytes16")(hash="identity")


@pytest.mark.parametrize("k", [1, 100, 1000])
@pytest.mark.parametrize("nvals", [1, 3, 50])
def test_wide_set_mode_degenerate_hash(cuda, k, nvals):
    """Set mode with a hash of very few values (round 6): the bucketed merge's buckets overflow and the
    sort-based merge takes over.  Set mode keeps the bottom-k by (scrambled hash, key words as
    unsigned 64-bit, word 0 first) -- computed here from the oracle's scramble."""
    import torch

    from oracle import oracle as O
    from reservoir_amd import Sampler

    n, width = 200_000, 16
    ids = _stream(n, 31 * k + nvals)
    rows = _rows(ids, width)
    hs = (np.asarray(ids, dtype=np.int64) % nvals) * 1000003 - 7
    ref = O.Distinct(k, 21, O.HASH_IDENTITY)
    r0, r1 = ref.r0, ref.r1
    sh = {int(x): O.scramble(r0, r1, int(x)) for x in np.unique(hs).tolist()}
    uniq = {}
    for r, h in zip(rows, hs.tolist()):
        b = bytes(r)
        uniq[b] = sh[h]
    words = lambda b: tuple(int.from_bytes(b[8 * w: 8 * w + 8], "little") for w in range(width // 8))
    want = sorted(sorted(uniq.items(), key=lambda kv: (kv[1], words(kv[0])))[:k], key=lambda kv: kv[0])
    d = Sampler.distinct(k, key_type=f"bytes{width}", seed=21, order="set")(hash=lambda b: 0)
    rd, hd = torch.from_numpy(rows).to(cuda), torch.from_numpy(hs).to(cuda)
    d.sample_all(rd[: n // 4], hashes=hd[: n // 4])
    d.sample_all(rd[n // 4:], hashes=hd[n // 4:])
    assert _sorted_rows(d.result()) == [kv[0] for kv in want]
