"""Multi-GPU sharding of the check.

Verdicts are per (key group, key range) and combine by OR, so the window
shards with no data-path exchange; the one collective is the verdict merge.

* :class:`KeyRangeShards` -- range partition of the key space of the window
  (configs 2 / 5: one index).  Every probe goes to each shard whose key range
  its ``[lo, hi]`` overlaps; routing is exact because a probe sent to a shard
  that holds none of its keys cannot conflict there, and every key lives in
  exactly one shard.
* :class:`GroupShards` -- (table, index, key length) groups assigned to ranks
  by size-balanced greedy (LPT), the north star's "(table, ix) hash"
  refined for balance (config 3).
* Table-lock probes need the table-wide max commit LSN: ranks merge their
  per-table maxima once per window build (:func:`allreduce_table_max`) and
  rank 0 evaluates the lock probes.
* :func:`merge_verdicts` -- ``all_reduce(MAX)`` on verdict bytes (= bitwise OR;
  RCCL has no OR op), then the bitmap is packed on the GPU.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import formats as F


def _leq(rows: np.ndarray, b: Sequence[int]) -> np.ndarray:
    """rows [W][n] (u64 words) <= b lexicographically."""
    lt = np.zeros(rows.shape[1], dtype=bool)
    eq = np.ones(rows.shape[1], dtype=bool)
    for j in range(rows.shape[0]):
        bj = np.uint64(b[j])
        lt |= eq & (rows[j] < bj)
        eq &= rows[j] == bj
    return lt | eq


def _geq(rows: np.ndarray, b: Sequence[int]) -> np.ndarray:
    gt = np.zeros(rows.shape[1], dtype=bool)
    eq = np.ones(rows.shape[1], dtype=bool)
    for j in range(rows.shape[0]):
        bj = np.uint64(b[j])
        gt |= eq & (rows[j] > bj)
        eq &= rows[j] == bj
    return gt | eq


def key_words(key: bytes, W: int) -> List[int]:
    b = bytes(key) + bytes(8 * W - len(key))
    return [int.from_bytes(b[8 * j:8 * j + 8], "big") for j in range(W)]


class KeyRangeShards:
    """world contiguous key ranges [lo_r, hi_r] (as W key words)."""

    def __init__(self, bounds: Sequence[Tuple[Sequence[int], Sequence[int]]]):
        self.bounds = [(list(a), list(b)) for a, b in bounds]
        self.world = len(self.bounds)

    @staticmethod
    def int64_uniform(world: int, value_bits: int, W: int) -> "KeyRangeShards":
        """Rank r owns int64 values [r << value_bits, (r+1) << value_bits)."""
        return KeyRangeShards([(key_words(F.enc_int64(r << value_bits), W),
                                key_words(F.enc_int64(((r + 1) << value_bits) - 1), W))
                               for r in range(world)])

    @staticmethod
    def int64_spans(world: int, span: int, W: int) -> "KeyRangeShards":
        """Rank r owns int64 values [r * span, (r+1) * span)."""
        return KeyRangeShards([(key_words(F.enc_int64(r * span), W),
                                key_words(F.enc_int64((r + 1) * span - 1), W))
                               for r in range(world)])

    def range_mask(self, m: dict, rank: int) -> np.ndarray:
        lo_b, hi_b = self.bounds[rank]
        return _leq(m["lo"], hi_b) & _geq(m["hi"], lo_b)

    def lock_mask(self, m: dict, rank: int) -> np.ndarray:
        return np.full(m["n_lock"], rank == 0, dtype=bool)


class GroupShards:
    """Key groups -> ranks by longest-processing-time greedy on group size."""

    def __init__(self, group_sizes: Dict[int, int], world: int):
        self.world = world
        load = [0] * world
        self.owner: Dict[int, int] = {}
        for g, sz in sorted(group_sizes.items(), key=lambda kv: (-kv[1], kv[0])):
            r = int(np.argmin(load))
            self.owner[g] = r
            load[r] += sz
        self.load = load

    def range_mask(self, m: dict, rank: int) -> np.ndarray:
        lut = np.zeros(max(self.owner, default=0) + 1, dtype=np.int64)
        for g, r in self.owner.items():
            lut[g] = r
        gid = np.asarray(m["gid"], dtype=np.int64)
        owner = np.where(gid < len(lut), lut[np.minimum(gid, len(lut) - 1)], 0)
        return owner == rank

    def lock_mask(self, m: dict, rank: int) -> np.ndarray:
        return np.full(m["n_lock"], rank == 0, dtype=bool)


def route(m: dict, range_mask: np.ndarray, lock_mask: np.ndarray) -> dict:
    """The sub-batch of a marshalled batch a rank probes."""
    idx = np.nonzero(range_mask)[0]
    lk = np.nonzero(lock_mask)[0]
    return dict(words=m["words"], n=len(idx), n_lock=len(lk), n_txn=m["n_txn"],
                lo=np.ascontiguousarray(m["lo"][:, idx]), hi=np.ascontiguousarray(m["hi"][:, idx]),
                gid=m["gid"][idx], snap=m["snap"][idx], txn=m["txn"][idx],
                lock_table=m["lock_table"][lk], lock_snap=m["lock_snap"][lk],
                lock_txn=m["lock_txn"][lk], forced=m["forced"])


def allreduce_table_max(table_max: np.ndarray, group=None) -> np.ndarray:
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(table_max.astype(np.int64))  # LSNs < 2^63
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.cpu().numpy().astype(np.uint64)


def merge_verdicts(verdict, group=None) -> None:
    """In-place OR of per-shard verdict bytes across ranks."""
    import torch.distributed as dist
    dist.all_reduce(verdict, op=dist.ReduceOp.MAX, group=group)
