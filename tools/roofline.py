"""VALU roofline of the Philox-bound kernels (K1 single stream, K2 segmented): algorithmic work and
the gfx950 issue peak it is priced against.

Neither kernel streams the keys -- a draw is a function of (seed, stream, index), so only the k
winning keys are read -- which makes them integer-VALU bound, not HBM bound.  The roofline:

  algorithmic work   level-0 Philox calls (one per 16-index block of [k, n)) + level-1 Philox calls
                     (one per index whose level-0 byte leaves j_i < k possible AND undetermined:
                     b_i (i+1) < 256 k, and for i < 256 the byte's interval [b, b+1) (i+1) / 256
                     straddles an integer -- otherwise j_i = floor(b_i (i+1) / 256) needs no level 1).
                     Work the kernels do beyond this (recomputes, queue traffic, masks) is overhead
                     and is NOT credited.
  issue cost         cycles per wave-instruction on one SIMD, measured with tools/micro_valu.hip under
                     rocprofv3 --pmc (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs / SQ_INSTS_VALU; 8 waves per
                     SIMD; profiles/r02/valu_costs.json): 4 cycles for every integer op used, the
                     64-bit v_mad_u64_u32 included (4.02-4.09 sustained in Philox-only loops):
                       level-0 call (counter words 1..3 wave-uniform): 18 v_mad_u64_u32 + 17 v_bitop3
                                                                       + 2 v_xor   (ISA of K1's loop)
                       level-1 call (full Philox4x32-10):             20 v_mad_u64_u32 + 20 v_bitop3
  peak               256 CU x 4 SIMD at the 2.4 GHz maximum clock (MI355X_MICROARCH.md), 64 lanes per
                     wave-instruction: peak calls/s = 1024 x 2.4e9 x 64 / (weighted cycles per wave-call)
  frac               achieved calls/s / peak calls/s (= algorithmic SIMD-cycles / (time x 1024 x 2.4e9))
"""
from __future__ import annotations

import json
import math
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COSTS_PATH = os.path.join(ROOT, "profiles", "r02", "valu_costs.json")
SIMDS = 256 * 4
CLOCK_HZ = 2.4e9
# measured on MI355X (profiles/r02/valu_costs.json "model"): one wave64 integer VALU instruction per
# 4 cycles per SIMD, whatever the op
_CYCLES = 4.0


def costs() -> dict:
    cyc, src = _CYCLES, "profiles/r02/valu_costs.json (model: 4 cycles per wave64 VALU instruction)"
    try:
        with open(COSTS_PATH) as f:
            cyc = float(json.load(f)["model"]["cycles_per_wave_instr"])
    except (OSError, KeyError, ValueError):
        src = "built-in 4 cycles per wave64 VALU instruction (profiles/r02/valu_costs.json absent)"
    c = {op: cyc for op in ("v_mad_u64_u32", "v_bitop3_b32", "v_xor_b32")}
    c["_source"] = src
    return c


def cycles_level0(c: dict) -> float:
    return 18 * c["v_mad_u64_u32"] + 17 * c["v_bitop3_b32"] + 2 * c["v_xor_b32"]


def cycles_level1(c: dict) -> float:
    return 20 * c["v_mad_u64_u32"] + 20 * c["v_bitop3_b32"]


def _level1_needed(i: np.ndarray, k: int) -> np.ndarray:
    """Expected number of level-1 calls at indices i (vector), draw format R2."""
    i = i.astype(np.float64)
    p = np.minimum(256.0, np.ceil(256.0 * k / (i + 1.0))) / 256.0
    return p


def _level1_small(k: int, lo: int, hi: int) -> float:
    """Exact expectation for indices < 256 (the byte may fix j_i by itself)."""
    tot = 0
    for i in range(max(lo, k), min(hi, 256)):
        for b in range(256):
            jmin = (b * (i + 1)) >> 8  # U = b 2^56
            jmax = ((((b + 1) << 56) - 1) * (i + 1)) >> 64  # U = (b + 1) 2^56 - 1
            tot += jmin < k and jmin != jmax
    return tot / 256.0


def k1_calls(n: int, k: int, i0: int = 0) -> tuple[float, float]:
    """(level-0 calls, expected level-1 calls) of K1 over global indices [max(i0, k), i0 + n)."""
    lo, hi = max(i0, k), i0 + n
    if hi <= lo:
        return 0.0, 0.0
    level0 = float(((hi + 15) >> 4) - (lo >> 4))
    dense_hi = min(hi, 256 * k)  # i + 1 < 256 k: more than the zero byte can hit
    level1 = _level1_small(k, lo, hi)
    a = max(lo, 256)
    step = 1 << 24
    while a < dense_hi:
        b = min(dense_hi, a + step)
        level1 += float(_level1_needed(np.arange(a, b, dtype=np.int64), k).sum())
        a = b
    level1 += max(0, hi - max(lo, 256 * k)) / 256.0  # sparse region: b_i == 0 only
    return level0, level1


def k2_calls(S: int, L: int, k: int) -> tuple[float, float]:
    """(level-0, level-1) calls of K2 for S streams of L elements each."""
    l0, l1 = k1_calls(L, k)
    return S * l0, S * l1


def valu_roofline(level0: float, level1: float, seconds: float, kernel: str, note: str = "") -> dict:
    c = costs()
    cyc = level0 / 64.0 * cycles_level0(c) + level1 / 64.0 * cycles_level1(c)  # SIMD-cycles
    calls = level0 + level1
    peak = calls / (cyc / (SIMDS * CLOCK_HZ)) / 1e9
    achieved = calls / seconds / 1e9
    d = {"bound": "valu", "achieved": round(achieved, 1), "peak": round(peak, 1), "unit": "GPhilox/s",
         "frac": round(achieved / peak, 4), "kernel": kernel, "launch_avg_us": round(seconds * 1e6, 2),
         "philox_calls_per_launch": {"level0": int(level0), "level1": int(round(level1))},
         "cycles_per_wave_call": {"level0": round(cycles_level0(c), 1), "level1": round(cycles_level1(c), 1)},
         "issue_costs": c["_source"],
         "peak_model": "1024 SIMDs x 2.4 GHz x 64 lanes / weighted cycles per wave-call (tools/roofline.py)"}
    if note:
        d["note"] = note
    return d


if __name__ == "__main__":
    l0, l1 = k1_calls(1_000_000_000, 1024)
    print("C2", l0, l1, valu_roofline(l0, l1, 105e-6, "k1"))
    l0, l1 = k2_calls(1 << 20, 4096, 64)
    print("C3", l0 / (1 << 20), l1 / (1 << 20), valu_roofline(l0, l1, 2.79e-3, "k2"))
    print(math.isfinite(l1))
