"""rsv_set_resolve_stream: each batch's slot resolve + publication forked onto a second stream after
its K1 (bench.py's pipelined steps).  Results must equal the oracle's last writers with several
samplers in flight on one stream, across a sampler's consecutive batches (the next batch's K1 waits
for the forked resolve: it reuses the winner table), and when the handle moves to another stream
(rsv_set_stream covers the forked work)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_pipelined_samplers_with_resolve_stream(cuda, oracle):
    import torch

    from reservoir_amd import Sampler

    n, k = (1 << 27) + 4099, 1024  # above the fused K1 + resolve limit (2^27 draws)
    keys = torch.arange(n, dtype=torch.int64, device=cuda) * 7 + 3
    main = torch.cuda.current_stream(cuda).cuda_stream
    side = torch.cuda.Stream(device=cuda).cuda_stream
    win = oracle.algo_r_last_writers(11, 12, k, 0, n)
    want = win * 7 + 3
    live = []
    for _ in range(4):  # four samplers in flight, their resolves on the side stream
        s = Sampler(k, seed=11, stream_id=12)()
        s.set_stream(main)
        s.set_resolve_stream(side)
        s.sample_all(keys)
        live.append(s)
    for s in live:
        assert np.array_equal(s.result(), want)
    # one sampler, two batches: the second batch's K1 waits for the first batch's forked resolve
    s = Sampler(k, seed=11, stream_id=12)()
    s.set_stream(main)
    s.set_resolve_stream(side)
    cut = (1 << 27) + 1
    s.sample_all(keys[:cut])
    s.sample_all(keys[cut:])
    assert np.array_equal(s.result(), want)
    # moved to a third stream right after sampling: the hand-over orders the forked resolve first
    s = Sampler(k, seed=11, stream_id=12)()
    s.set_stream(main)
    s.set_resolve_stream(side)
    s.sample_all(keys)
    other = torch.cuda.Stream(device=cuda)
    s.set_stream(other.cuda_stream)
    idx, _, _, _ = s.export_state(cuda)
    torch.cuda.synchronize()
    assert np.array_equal(idx.cpu().numpy(), win)
    assert np.array_equal(s.result(), want)


@pytest.mark.parametrize("engine", ["philox_r", "java_l"])
def test_host_batches_with_resolve_stream(cuda, oracle, engine):
    """Host-memory batches over several device chunks (4 Mi keys each) with the resolve forked: the
    next chunk's copy into the engine's chunk buffer must wait for the previous resolve's reads
    (join before any write to the chunk)."""
    import torch

    from reservoir_amd import Sampler

    n, k = 3 * (1 << 22) + 12345, 4096
    keys = (np.arange(n, dtype=np.int64) * 13 + 5)
    side = torch.cuda.Stream(device=cuda).cuda_stream
    s = Sampler(k, engine=engine, seed=21, stream_id=3)()
    s.set_stream(torch.cuda.current_stream(cuda).cuda_stream)
    s.set_resolve_stream(side)
    s.sample_all(keys[:n // 2])
    s.sample_all(keys[n // 2:])
    got = s.result()
    if engine == "philox_r":
        want = oracle.algo_r_last_writers(21, 3, k, 0, n) * 13 + 5
    else:
        ref = oracle.AlgoL(k, 21)
        ref.sample_all(keys)
        want = ref.result()
    assert np.array_equal(got, want)


def test_dropped_device_batch_with_resolve_stream(cuda, oracle):
    """A device batch dropped right after sample_all: the caching allocator must not hand its memory
    to a new tensor while the forked resolve still reads it (the tensor is recorded on both streams)."""
    import torch

    from reservoir_amd import Sampler

    n, k = (1 << 27) + 77, 1024
    side = torch.cuda.Stream(device=cuda).cuda_stream
    s = Sampler(k, seed=5, stream_id=9)()
    s.set_stream(torch.cuda.current_stream(cuda).cuda_stream)
    s.set_resolve_stream(side)
    keys = torch.arange(n, dtype=torch.int64, device=cuda) * 3 + 1
    s.sample_all(keys)
    del keys
    junk = torch.full((n,), -7, dtype=torch.int64, device=cuda)  # may reuse the freed block
    want = oracle.algo_r_last_writers(5, 9, k, 0, n) * 3 + 1
    assert np.array_equal(s.result(), want)
    del junk
