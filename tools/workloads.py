"""Synthetic inputs of BASELINE.json's configs, generated on the device with torch.

Shared by bench.py, tools/bench_paths.py and the full-size parity tests (tests/test_gpu_configs.py).
torch int64 arithmetic wraps like Java Long; logical right shifts are emulated with a mask.

  splitmix_fill(out, base)      out[i] = splitmix64(base + i)                        (C1, C2, C3)
  c4_data(n, dev)               C4: D = 0.7 n distinct values v_j = splitmix64(j ^ 0xD15C); element
                                i takes v_i for i < D and v_{hash(i) mod D} otherwise (the 30 %
                                duplicates), hash(i) = splitmix64(i ^ 0xD0B) >>> 1; positions
                                shuffled by a 4-round Feistel permutation of [0, n) (seed 7,
                                cycle-walking)
  c4_slice(n, lo, hi, dev)      positions [lo, hi) of c4_data(n), generated directly (inverse
                                permutation): one rank's piece of C4's 8-way split
  hash_twins(keys, bits)        keys whose java.lang.Long.hashCode takes only 2^bits values (many
                                distinct keys per hash bucket: the ordered distinct path's replay)
  uuid_rows(vals, twin_bits)    16-byte UUID keys, one per distinct value (optionally hash twins)
  uuid_hash(rows)               java.util.UUID.hashCode of such rows
"""
from __future__ import annotations

import torch

_G = 0x9E3779B97F4A7C15 - (1 << 64)
_M1 = 0xBF58476D1CE4E5B9 - (1 << 64)
_M2 = 0x94D049BB133111EB - (1 << 64)


def _srl(z: torch.Tensor, s: int) -> torch.Tensor:
    """Logical right shift of int64 (Java >>>)."""
    return (z >> s) & ((1 << (64 - s)) - 1)


def smix(x: torch.Tensor) -> torch.Tensor:
    """splitmix64(x) elementwise (x as int64 bits)."""
    z = x + _G
    z = (z ^ _srl(z, 30)) * _M1
    z = (z ^ _srl(z, 27)) * _M2
    return z ^ _srl(z, 31)


def splitmix_fill(out: torch.Tensor, base: int, chunk: int = 1 << 27) -> None:
    """out[i] = splitmix64(base + i) (C2 base 0x5EED0000, C3 base 0)."""
    n = out.numel()
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        out[a:b] = smix(torch.arange(base + a, base + b, dtype=torch.int64, device=out.device))


def feistel_perm(n: int, seed: int, device, chunk: int = 1 << 26) -> torch.Tensor:
    """A bijection of [0, n): 4-round balanced Feistel network on 2h >= log2(n) bits, cycle-walked
    back into range."""
    bits = max(2, (n - 1).bit_length())
    bits += bits & 1
    h = bits // 2
    mask = (1 << h) - 1

    def enc(x):
        lo, hi = x & mask, x >> h
        for r in range(4):
            f = smix(lo + ((seed * 4 + r) << 40)) & mask
            lo, hi = hi ^ f, lo
        return (hi << h) | lo

    y = torch.empty(n, dtype=torch.int64, device=device)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        y[a:b] = enc(torch.arange(a, b, dtype=torch.int64, device=device))
    while True:
        bad = torch.nonzero(y >= n).flatten()
        if bad.numel() == 0:
            return y
        y[bad] = enc(y[bad])


def _feistel_params(n: int):
    bits = max(2, (n - 1).bit_length())
    bits += bits & 1
    h = bits // 2
    return h, (1 << h) - 1


def feistel_inverse(y: torch.Tensor, n: int, seed: int) -> torch.Tensor:
    """feistel_perm(n, seed)^-1 at the positions y: the rounds run backwards, and cycle-walking
    inverts by walking the inverse permutation until it lands inside [0, n)."""
    h, mask = _feistel_params(n)

    def dec(x):
        lo, hi = x & mask, x >> h
        for r in reversed(range(4)):  # enc round: (lo, hi) -> (hi ^ f(lo), lo)
            lo, hi = hi, lo ^ (smix(hi + ((seed * 4 + r) << 40)) & mask)
        return (hi << h) | lo

    x = dec(y)
    while True:
        bad = torch.nonzero(x >= n).flatten()
        if bad.numel() == 0:
            return x
        x[bad] = dec(x[bad])


def _c4_value(i: torch.Tensor, D: int) -> torch.Tensor:
    vi = torch.where(i < D, i, _srl(smix(i ^ 0xD0B), 1) % max(D, 1))
    return smix(vi ^ 0xD15C)


def c4_slice(n: int, lo: int, hi: int, device, dup: float = 0.3, seed: int = 7, chunk: int = 1 << 26,
             out: torch.Tensor | None = None) -> torch.Tensor:
    """Positions [lo, hi) of the C4 sequence of n keys (= c4_data(n)[lo:hi]) without building the
    whole sequence: position p holds value v_{perm^-1(p)}.  A rank of C4's 8-way split generates
    its own piece this way; the full 4e9 sequence is 8 such pieces."""
    D = int(round(n * (1.0 - dup)))
    if out is None:
        out = torch.empty(hi - lo, dtype=torch.int64, device=device)
    for a in range(lo, hi, chunk):
        b = min(hi, a + chunk)
        src = feistel_inverse(torch.arange(a, b, dtype=torch.int64, device=device), n, seed)
        out[a - lo:b - lo] = _c4_value(src, D)
    return out


def c4_data(n: int, device, dup: float = 0.3, seed: int = 7, chunk: int = 1 << 26) -> torch.Tensor:
    """C4: n Long keys, D = (1 - dup) n distinct values, Feistel-shuffled."""
    return c4_slice(n, 0, n, device, dup, seed, chunk)


def c4_data_scatter(n: int, device, dup: float = 0.3, seed: int = 7, chunk: int = 1 << 26) -> torch.Tensor:
    """The defining construction of c4_data (values scattered through the forward permutation);
    kept to check c4_slice against (tests/test_workloads.py)."""
    D = int(round(n * (1.0 - dup)))
    vals = torch.empty(n, dtype=torch.int64, device=device)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        vals[a:b] = _c4_value(torch.arange(a, b, dtype=torch.int64, device=device), D)
    perm = feistel_perm(n, seed, device)
    out = torch.empty_like(vals)
    out[perm] = vals
    return out


def hash_twins(keys: torch.Tensor, bits: int = 24) -> torch.Tensor:
    """(hi, lo) -> (hi, hi ^ (lo & (2^bits - 1))): Long.hashCode = hi ^ lo' = lo & (2^bits - 1)."""
    hi = _srl(keys, 32)
    lo = (hi ^ (keys & ((1 << bits) - 1))) & 0xFFFFFFFF
    return (hi << 32) | lo


def uuid_rows(vals: torch.Tensor, twin_bits: int | None = None) -> torch.Tensor:
    """16-byte keys (java.util.UUID laid out [mostSigBits | leastSigBits], little-endian Longs) as a
    (n, 16) uint8 tensor, one distinct row per distinct value v: [v, splitmix64(v ^ 0xAA)].  With
    twin_bits, [v, v ^ (v & (2^twin_bits - 1))] instead: UUID.hashCode = v & (2^twin_bits - 1), so
    ~n / 2^twin_bits distinct keys share each hash value (the ordered distinct path's replay)."""
    lo = smix(vals ^ 0xAA) if twin_bits is None else vals & ~((1 << twin_bits) - 1)
    return torch.stack([vals, lo], dim=1).contiguous().view(torch.uint8)


def uuid_hash(rows: torch.Tensor) -> torch.Tensor:
    """java.util.UUID.hashCode (.toLong) of (n, 16) uint8 rows, on the device."""
    w = rows.contiguous().view(torch.int64).view(-1, 2)
    hilo = w[:, 0] ^ w[:, 1]
    x = (_srl(hilo, 32) ^ hilo) & 0xFFFFFFFF
    return (x ^ 0x80000000) - 0x80000000
