"""Fixed-width byte keys (key_type "bytesN": UUIDs, composite keys) in the element sampler.

The sampler never looks inside a key, so a byte-key reservoir must hold exactly the keys at the
positions the oracle's Algorithm R (fed the same draws) selects: keys here are derived from their
position, and the expected rows are the same derivation applied to the oracle's winning positions.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rows(ids, width):
    """width-byte key of element id: the splitmix stream of the id, little-endian words."""
    ids = np.asarray(ids, dtype=np.uint64)
    words = width // 8
    out = np.empty((ids.size, words), dtype=np.uint64)
    for w in range(words):
        z = ids * np.uint64(0x9E3779B97F4A7C15) + np.uint64((w * 0x632BE59BD9B4E019 + 1) & (2**64 - 1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        out[:, w] = z ^ (z >> np.uint64(31))
    return out.view(np.uint8).reshape(ids.size, width)


@pytest.mark.parametrize("width", [16, 24, 64])
@pytest.mark.parametrize("k,n", [(1, 1000), (100, 50), (1024, 300_000), (9000, 120_000)])
def test_wide_keys_parity(cuda, oracle, width, k, n):
    import torch

    from reservoir_amd import Sampler

    ids = np.arange(n, dtype=np.int64)
    want_ids, _ = oracle.algo_r(77 + width, 5, k, ids)
    want = _rows(want_ids, width)
    keys = _rows(ids, width)
    s = Sampler(k, key_type=f"bytes{width}", seed=77 + width, stream_id=5)()
    s.sample_all(torch.from_numpy(keys).to(cuda))       # device rows
    got = s.result()
    assert got.shape == (min(n, k), width)
    assert np.array_equal(got, want[: min(n, k)])
    h = Sampler(k, key_type=f"bytes{width}", seed=77 + width, stream_id=5)()
    cut = n // 3
    h.sample_all(keys[:cut])                             # host rows, two batches
    for row in keys[cut: cut + 10]:                      # per-element sample()
        h.sample(row.tobytes())
    h.sample_all(keys[cut + 10:])
    assert np.array_equal(h.result(), want[: min(n, k)])


def test_wide_keys_split_merge(cuda, oracle):
    """Index-range split + packed merge with 32-byte keys (distributed.combine's rows)."""
    import torch

    from reservoir_amd import Sampler

    n, k, width, parts = 400_003, 512, 32, 3
    ids = np.arange(n, dtype=np.int64)
    want_ids, _ = oracle.algo_r(3, 4, k, ids)
    keys = torch.from_numpy(_rows(ids, width)).to(cuda)
    bounds = np.linspace(0, n, parts + 1).astype(np.int64)
    row_len = k * (1 + width // 8)
    rows = torch.zeros((parts - 1, row_len), dtype=torch.int64, device=cuda)
    for p in range(parts - 1):
        s = Sampler(k, key_type=f"bytes{width}", seed=3, stream_id=4)()
        s.seek(int(bounds[p]))
        s.sample_all(keys[bounds[p]:bounds[p + 1]])
        s.export_packed(rows[p])
    last = Sampler(k, key_type=f"bytes{width}", seed=3, stream_id=4)()
    last.seek(int(bounds[-2]))
    last.sample_all(keys[bounds[-2]:])
    last.merge_packed(rows, n)
    assert np.array_equal(last.result(), _rows(want_ids, width))


def test_wide_keys_rejected_where_unsupported(cuda):
    from reservoir_amd import IllegalArgumentException, Sampler

    with pytest.raises(IllegalArgumentException):
        Sampler(10, key_type="bytes12")()
    s = Sampler(4, key_type="bytes16")()
    with pytest.raises(IllegalArgumentException):
        s.sample(b"short")
