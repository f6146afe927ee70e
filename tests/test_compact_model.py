"""CPU check of the compact-code bound mapping (hsc_compact.hip header):
for random groups of keys with few varying bits and random probe bounds,
#rows < X == #codes < lo'(X) and #rows <= X == #codes <= hi'(X), with
lo' / hi' computed by the rules the kernel implements (restated here over
Python integers, independently of the device bit tricks)."""
import numpy as np
import pytest


def _code(x, V):
    c = 0
    for p in V:
        c = (c << 1) | ((x >> p) & 1)
    return c


def bound(x, C, M, nbits, V, kind):
    """kind 1: lo' (count codes < lo'), 2: hi' (count codes <= hi'); None =
    the range misses every row."""
    d = (x ^ C) & ~M & ((1 << nbits) - 1)
    nv = len(V)
    if d == 0:
        return _code(x, V)
    b = d.bit_length() - 1                  # first mismatch at a constant bit
    Vp = [p for p in V if p > b]            # varying positions before it
    prefix, npb, k = _code(x, Vp), len(Vp), nv - len(Vp)
    xb = (x >> b) & 1
    if kind == 1:
        if xb:
            if prefix + 1 >= (1 << npb):
                return None                 # above every row
            return (prefix + 1) << k
        return prefix << k
    if xb:
        return (prefix << k) | ((1 << k) - 1)
    if prefix == 0:
        return None                         # below every row
    return ((prefix - 1) << k) | ((1 << k) - 1)


@pytest.mark.parametrize("seed", range(20))
def test_bound_mapping_counts(seed):
    rng = np.random.default_rng(seed)
    W = int(rng.integers(1, 4))
    nbits = 64 * W
    base = int.from_bytes(rng.integers(0, 256, size=8 * W, dtype=np.uint8).tobytes(), "big")
    vm = 0
    for _ in range(int(rng.integers(1, 24))):
        vm |= 1 << int(rng.integers(0, nbits))
    rows = sorted({(base & ~vm) | (int.from_bytes(rng.integers(0, 256, size=8 * W, dtype=np.uint8)
                                                  .tobytes(), "big") & vm)
                   for _ in range(int(rng.integers(1, 60)))})
    C, M = rows[0], 0
    for r in rows:
        M |= r ^ C
    V = [p for p in range(nbits - 1, -1, -1) if (M >> p) & 1]
    codes = [_code(r, V) for r in rows]
    assert codes == sorted(codes) and len(set(codes)) == len(codes)
    for _ in range(300):
        u = rng.random()
        if u < 0.3:
            x = rows[int(rng.integers(0, len(rows)))]
        else:
            x = rows[int(rng.integers(0, len(rows)))]
            for _ in range(int(rng.integers(1, 4))):
                x ^= 1 << int(rng.integers(0, nbits))
            if u > 0.9:
                x = int(rng.integers(0, 2)) * ((1 << nbits) - 1)
        lt = sum(r < x for r in rows)
        le = sum(r <= x for r in rows)
        lo = bound(x, C, M, nbits, V, 1)
        hi = bound(x, C, M, nbits, V, 2)
        if lo is None:
            assert lt == len(rows)
        else:
            assert lt == sum(c < lo for c in codes)
        if hi is None:
            assert le == 0
        else:
            assert le == sum(c <= hi for c in codes)
