"""The byte-row RandomValues oracle (oracle.DistinctRows, oracle.c or_drows_*) pinned against the
Long oracle (oracle.Distinct, itself pinned by KATs and the reference's test properties): one-word
rows whose precomputed hash is the Long's own hash must give the SAME sequential state -- element
set, heap ties included -- as Sampler.distinct over the Longs (Sampler.scala:394-409).  CPU only."""
import numpy as np
import pytest


def _long_hashcode(v):
    v = v.astype(np.int64)
    x = (v ^ ((v >> 32) & 0xFFFFFFFF)) & 0xFFFFFFFF
    return ((x ^ 0x80000000) - 0x80000000).astype(np.int64)  # (int) cast, widened


@pytest.mark.parametrize("k", [1, 7, 100, 2000])
@pytest.mark.parametrize("hash_kind", ["identity", "java_long"])
def test_rows_oracle_equals_long_oracle(oracle, k, hash_kind):
    rng = np.random.default_rng(k)
    vals = rng.integers(-2**63, 2**63 - 1, size=40_000, dtype=np.int64)
    if hash_kind == "java_long":  # few hash values: the boundary bucket ties, heap order decides
        vals = (vals & ~0xFFFFFFFF) | ((vals >> 32) ^ rng.integers(0, 500, size=vals.size)) & 0xFFFFFFFF
    vals = np.concatenate([vals, vals[rng.integers(0, vals.size, 15_000)]])
    kind = oracle.HASH_IDENTITY if hash_kind == "identity" else oracle.HASH_JAVA_LONG
    ref = oracle.Distinct(k, 5, kind)
    ref.sample_all(vals)
    want_k, want_h = ref.result()
    rows = oracle.DistinctRows(k, 5, 8)
    hashes = vals if hash_kind == "identity" else _long_hashcode(vals)
    rows.sample_all(vals.view(np.uint8).reshape(-1, 8), hashes)
    got_rows, got_h = rows.result()
    got = np.sort(got_rows.view(np.int64).reshape(-1))
    assert np.array_equal(np.sort(got_h), np.sort(want_h))
    assert np.array_equal(got, np.sort(want_k))


def test_rows_oracle_dedups_by_every_word(oracle):
    """Keys equal in their first word but not the second are distinct; equal rows are one element."""
    k = 50
    base = np.arange(40, dtype=np.uint64)
    rows = np.zeros((80, 2), dtype=np.uint64)
    rows[:40, 0] = base
    rows[40:, 0] = base
    rows[40:, 1] = 1  # same first word, different second
    rows = np.concatenate([rows, rows[:10]])  # exact repeats
    d = oracle.DistinctRows(k, 1, 16)
    d.sample_all(rows.view(np.uint8), np.zeros(rows.shape[0], dtype=np.int64))  # one hash for all
    got, _ = d.result()
    assert got.shape[0] == 50  # 80 distinct keys, k = 50 of them
    assert len({bytes(r) for r in got}) == 50


def test_uuid_hashcode_matches_jdk_formula(oracle):
    # UUID.hashCode: hilo = msb ^ lsb; (int)(hilo >> 32) ^ (int) hilo
    for msb, lsb in [(0, 0), (1, 2), (0x123456789ABCDEF0, 0x0FEDCBA987654321), (-1, 5)]:
        hilo = (msb ^ lsb) & (2**64 - 1)
        v = ((hilo >> 32) ^ hilo) & 0xFFFFFFFF
        want = v - 2**32 if v >= 2**31 else v
        assert oracle.uuid_hashcode(msb, lsb) == want
