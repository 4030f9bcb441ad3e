"""Generate tests/golden/golden.json from the CPU oracle (oracle/oracle.c).

The reference (Scala 2.13 + sbt) cannot be built or run in this image (no JVM, no jars, no
network), so these vectors are restatement-derived.  They are pinned by:
  * published java.util.Random known answers and Random123 Philox KATs (tests/test_oracle_kats.py);
  * the survey's independently restated vector (k=20 over 1..3000, Random(0)),
    which the "survey_k20" case must reproduce;
  * the reference's own test properties (sample == sampleAll over every collection shape,
    SamplerTest.scala:117-142), checked in tests/test_oracle_reference_props.py.
Run:  python tests/golden/gen_golden.py   (rewrites golden.json deterministically)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402


def algo_l_case(k, n, seed):
    s = O.AlgoL(k, seed)
    s.sample_all(np.arange(1, n + 1, dtype=np.int64))
    pos, slot = s.events()
    return {"k": k, "n": n, "seed": seed, "elements": "1..n", "result": s.result().tolist(),
            "n_events": int(pos.size), "events_head": [[int(p), int(q)] for p, q in zip(pos[:16], slot[:16])]}


def draws_case(seed, stream, i0, n):
    return {"seed": seed, "stream": stream, "i0": i0, "n": n,
            "j": [int(x) for x in O.export_draws(seed, stream, i0, n)],
            "u": [int(O.draw_u64(seed, stream, i0 + t)) for t in range(n)]}


def algo_r_case(seed, stream, k, n, key_base):
    keys = O.splitmix_keys(key_base, n)
    res, repl = O.algo_r(seed, stream, k, keys)
    return {"seed": seed, "stream": stream, "k": k, "n": n, "key_base": key_base,
            "result": res.tolist(), "replacements": int(repl)}


def distinct_case(k, seed, hash_kind, values):
    d = O.Distinct(k, seed, hash_kind)
    d.sample_all(values)
    keys, hs = d.result()
    return {"k": k, "seed": seed, "hash_kind": hash_kind, "values": [int(v) for v in values],
            "r0": d.r0, "r1": d.r1, "result_sorted_by_hash": keys.tolist(), "hashes": hs.tolist()}


def main():
    rng = np.random.default_rng(2024)
    g = {
        "survey_k20": algo_l_case(20, 3000, 0),
        "algo_l": [algo_l_case(5, 10, 0), algo_l_case(100, 100_000, 42), algo_l_case(64, 10_000, 7),
                   algo_l_case(1000, 50_000, 123), algo_l_case(1, 1000, 9), algo_l_case(3, 3, 1)],
        "draws": [draws_case(0, 0, 0, 48), draws_case(0xC0FFEE, 0x5A5A, 1000, 32),
                     draws_case(1, 2, 2**32 - 7, 16), draws_case(2**63 + 5, 2**40 + 3, 2**40, 16)],
        "algo_r": [algo_r_case(0xC0FFEE, 0, 64, 5000, 0x5EED0000), algo_r_case(7, 3, 5, 10, 1),
                   algo_r_case(11, 0, 1000, 20_000, 99), algo_r_case(0, 0, 1, 777, 5)],
        "distinct": [
            distinct_case(10, 0, O.HASH_JAVA_INT, [1] * 10),
            distinct_case(5, 0, O.HASH_JAVA_INT, list(range(1, 11))),
            distinct_case(50, 0, O.HASH_IDENTITY,
                          [int(x) for x in rng.integers(-2**63, 2**63 - 1, size=300, dtype=np.int64)] * 2),
            distinct_case(20, 77, O.HASH_JAVA_LONG, [int(x) for x in rng.integers(0, 40, size=200)]),
        ],
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
