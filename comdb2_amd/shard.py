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


# ---- config 4: dependency graph + SCC sharded by key -----------------------
# Every WW / WR / RW edge belongs to one key (hsc_graph.hip), so a history
# split by key gives each rank an exact part of the edge set with no
# exchange.  Cycles need a backward (src > dst in commit order) edge and stay
# inside the intervals [dst, src] of backward edges, so the ranks OR their
# "covers" (all_reduce MAX over u8 per txn), all-gather only their edges
# between covered txns, and every rank colours that small graph
# (include/hip_serial.h, hsc_dep_graph_build / _cover / _cut / _scc_cut).

def key_owner(key: np.ndarray, world: int) -> np.ndarray:
    """Rank owning each history key (Fibonacci hash of the key, mod world)."""
    h = (np.asarray(key, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(32)
    return (h % np.uint64(world)).astype(np.int64)


def history_shard(h, rank: int, world: int):
    """The ops of a History whose key this rank owns (order kept; txn ids and
    ntxn stay global)."""
    from .workloads import History
    if world == 1:
        return h
    sel = key_owner(h.key, world) == rank
    return History(h.txn[sel], h.key[sel], h.is_write[sel], h.observed[sel], h.ntxn)


class DeviceHistory:
    """A History's ops resident on a GPU (torch tensors: txn i32, key i64,
    is_write u8, observed i32 with -1 = initial version)."""

    def __init__(self, h, device):
        import torch
        self.ntxn, self.nops = int(h.ntxn), int(len(h.txn))
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        self.txn = up(np.asarray(h.txn, np.uint32).view(np.int32))
        self.key = up(np.asarray(h.key, np.uint64).view(np.int64))
        self.is_write = up(np.asarray(h.is_write, np.uint8))
        self.observed = up(np.asarray(h.observed, np.int64).astype(np.int32))


def device_history(h, device) -> DeviceHistory:
    return DeviceHistory(h, device)


class GpuGraph:
    """The sharded-SCC steps of a Validator over torch tensors on its GPU.
    Every call synchronises torch's stream first (the library runs on its
    own stream and returns after synchronising it)."""

    def __init__(self, validator, device, full: bool = False):
        self.v, self.device, self.full = validator, device, full

    def _sync(self):
        import torch
        torch.cuda.synchronize(self.device)

    def build(self, h) -> dict:
        if isinstance(h, DeviceHistory):
            self._sync()
            return self.v.dep_graph_build_device(h.nops, h.ntxn, h.txn.data_ptr(), h.key.data_ptr(),
                                                 h.is_write.data_ptr(), h.observed.data_ptr(),
                                                 self.full)
        return self.v.dep_graph_build(h, self.full)

    def cover(self, cover) -> None:
        self._sync()
        self.v.dep_graph_cover(cover.data_ptr())

    def cut(self, cover):
        import torch
        self._sync()
        m = self.v.dep_graph_cut(cover.data_ptr())
        rows = torch.empty(max(m, 1), dtype=torch.int64, device=self.device)
        self._sync()
        self.v.dep_graph_cut(cover.data_ptr(), rows.data_ptr(), m)
        return rows[:m]

    def scc_cut(self, ntxn: int, cover, rows, scc) -> dict:
        self._sync()
        return self.v.dep_graph_scc_cut(ntxn, cover.data_ptr(), rows.data_ptr(), rows.numel(),
                                        scc.data_ptr())


def sharded_scc(graph, h_shard, ntxn: int, device, group=None):
    """scc[ntxn] (int32 tensor on `device`: largest txn of each txn's
    component, identical on every rank) of the union of the ranks' history
    shards, plus per-step stats.  `graph` is a GpuGraph (or a model with the
    same four methods)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    st = {"build": graph.build(h_shard)}
    cover = torch.zeros(max(ntxn, 1), dtype=torch.uint8, device=device)
    graph.cover(cover)
    # gloo (CPU rehearsal of the N > 1 path) exchanges host copies
    cd = device if world == 1 or dist.get_backend(group) == "nccl" else torch.device("cpu")
    if world > 1:
        c = cover.to(cd)
        dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
        cover = c.to(device)
    rows = graph.cut(cover)
    st["cut_rows_local"] = int(rows.numel())
    if world > 1:
        n = torch.tensor([rows.numel()], dtype=torch.int64, device=cd)
        sizes = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(sizes, n, group=group)
        mx = max(1, max(int(x.item()) for x in sizes))
        pad = torch.full((mx,), -1, dtype=torch.int64, device=cd)  # ~0 rows: padding
        pad[: rows.numel()] = rows.to(cd)
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        rows = torch.cat(parts).to(device)
    st["cut_rows"] = int(rows.numel())
    scc = torch.empty(max(ntxn, 1), dtype=torch.int32, device=device)
    st["scc"] = graph.scc_cut(ntxn, cover, rows, scc)
    return scc[:ntxn], st
