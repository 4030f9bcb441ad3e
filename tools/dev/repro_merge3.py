"""Dev repro: identity-hash distinct merge of 3 pieces, in one process (merge_local) and element-wise
diagnostics vs the oracle (round-3 investigation of test_gloo_ranks_real_engine[3])."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle as O  # noqa: E402
from reservoir_amd import Sampler  # noqa: E402
from reservoir_amd import distributed as D  # noqa: E402

dev = torch.device("cuda", 0)
vals = np.random.default_rng(3).integers(-2**63, 2**63 - 1, size=400_000, dtype=np.int64)
vals = np.concatenate([vals, vals[: 150_000]])
ref = O.Distinct(5000, 9, O.HASH_IDENTITY)
ref.sample_all(vals)
want = set(ref.result()[0].tolist())
for world in (2, 3, 4):
    ss = []
    for r in range(world):
        lo, hi = D.shard_range(vals.size, r, world)
        s = Sampler.distinct(5000, seed=9)(hash="identity")
        s.sample_all(torch.from_numpy(vals[lo:hi]).to(dev))
        ss.append(s)
    for into in (0, None):
        t = ss[0] if into == 0 else Sampler.distinct(5000, seed=9)(hash="identity")
        if into == 0:
            ss2 = []
            for r in range(world):
                lo, hi = D.shard_range(vals.size, r, world)
                s = Sampler.distinct(5000, seed=9)(hash="identity")
                s.sample_all(torch.from_numpy(vals[lo:hi]).to(dev))
                ss2.append(s)
            t = ss2[0]
            D.merge_local(t, ss2)
        else:
            D.merge_local(t, ss)
        got = set(t.result().tolist())
        print(f"world={world} into_shard0={into == 0}: equal={got == want} |got|={len(got)} "
              f"missing={len(want - got)} extra={len(got - want)}", flush=True)
