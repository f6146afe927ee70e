"""Multi-GPU sharding of the check.

Verdicts are per (key group, key range) and combine by OR, so the window
shards with no data-path exchange; the one collective is the verdict merge.

* :class:`KeyRangeShards` -- range partition of the key space of the window
  (configs 2 / 5: one index).  Every probe goes to each shard whose key range
  its ``[lo, hi]`` overlaps; routing is exact because a probe sent to a shard
  that holds none of its keys cannot conflict there, and every key lives in
  exactly one shard.
* :class:`GroupShards` -- (table, index, key length) groups assigned to ranks
  by work-balanced greedy (LPT), the north star's "(table, ix) hash"
  refined for balance (config 3); a hot group is first cut into key-range
  pieces, so one (table, index) cannot cap the scaling.
* Table-lock probes need the table-wide max commit LSN: ranks merge their
  per-table maxima once per window build (:func:`allreduce_table_max`) and
  rank 0 evaluates the lock probes.
* Verdict merge: every rank packs its shard's verdicts into a bitmap on the
  GPU, one all-gather of the N bitmaps (:func:`gather_bitmaps`: RCCL has no
  bitwise-OR reduction) and an OR of the N parts on the GPU
  (``hsc_or_bitmaps``).  :func:`merge_verdicts` (``all_reduce(MAX)`` on
  verdict bytes) is the host-side equivalent the gloo rehearsals use.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

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

    @staticmethod
    def int64_splitters(splitters: Sequence[int], W: int) -> "KeyRangeShards":
        """Rank j owns int64 values [splitters[j-1], splitters[j]); the first
        and last ranks own everything below / above (any key bytes)."""
        sp = [int(x) for x in splitters]
        world = len(sp) + 1
        b = []
        for r in range(world):
            lo = [0] * W if r == 0 else key_words(F.enc_int64(sp[r - 1]), W)
            # the upper bound padded with 0xFF: every key that has it as a prefix
            hi = ([(1 << 64) - 1] * W if r == world - 1
                  else key_words(F.enc_int64(sp[r] - 1) + b"\xff" * (8 * W - 9), W))
            b.append((lo, hi))
        return KeyRangeShards(b)

    def range_mask(self, m: dict, rank: int) -> np.ndarray:
        lo_b, hi_b = self.bounds[rank]
        return _leq(m["lo"], hi_b) & _geq(m["hi"], lo_b)

    def lock_mask(self, m: dict, rank: int) -> np.ndarray:
        return np.full(m["n_lock"], rank == 0, dtype=bool)


def _lex_order(words: np.ndarray) -> np.ndarray:
    """Order of the columns of words [W][n] in lexicographic (memcmp) order."""
    return np.lexsort(words[::-1]) if words.shape[1] else np.zeros(0, np.int64)


class GroupShards:
    """Key groups -> ranks by longest-processing-time greedy (LPT) on each
    group's probe work (rows + RANGE_COST x ranges, SURVEY.md §7 hard part 5).
    A group heavier than total / (2 world) -- the one hot (table, index) of a
    skewed schema, whose weight alone would cap the speedup -- is first cut
    into key-range pieces at weighted quantiles of its rows and range lower
    bounds (split_keys), each no heavier than that; a piece owns the group's
    keys in [lo, hi) (as key words), every row lives in one piece, and a range
    goes to each piece of its group that it overlaps (exact, as for
    KeyRangeShards: a piece holding none of a range's keys cannot conflict).

    group_load: {gid: work}; split_keys: {gid: (words u64[W][n], weights
    f64[n])} for the groups that may be split (rows and range lower bounds of
    the group, any order).  owner: {gid: rank} of the unsplit groups; pieces:
    [(gid, lo words or None, hi words or None, rank, load)]."""

    def __init__(self, group_load: Dict[int, float], world: int,
                 split_keys: Optional[Dict[int, Tuple[np.ndarray, np.ndarray]]] = None):
        self.world = world
        total = float(sum(group_load.values()))
        cap = total / (2 * world) if world > 1 else float("inf")
        items = []  # (load, gid, lo, hi)
        for g, ld in group_load.items():
            k = int(np.ceil(ld / cap)) if ld > cap and split_keys and g in split_keys else 1
            bounds = self._cut(*split_keys[g], k) if k > 1 else []
            if not bounds:
                items.append((float(ld), g, None, None))
                continue
            words, wts = split_keys[g]
            edges = [None] + bounds + [None]
            for lo, hi in zip(edges[:-1], edges[1:]):
                m = np.ones(words.shape[1], bool)
                if lo is not None:
                    m &= _geq(words, lo)
                if hi is not None:
                    m &= ~_geq(words, hi)
                share = float(wts[m].sum()) / max(float(wts.sum()), 1e-30)
                items.append((ld * share, g, lo, hi))
        load = [0.0] * world
        self.pieces = []
        for ld, g, lo, hi in sorted(items, key=lambda it: (-it[0], it[1],
                                                           [] if it[2] is None else it[2])):
            r = int(np.argmin(load))
            self.pieces.append((g, lo, hi, r, ld))
            load[r] += ld
        self.load = load
        self.owner: Dict[int, int] = {g: r for g, lo, hi, r, _ in self.pieces
                                      if lo is None and hi is None}
        self.split: Dict[int, list] = {}
        for g, lo, hi, r, _ in self.pieces:
            if lo is not None or hi is not None:
                self.split.setdefault(g, []).append((lo, hi, r))

    @staticmethod
    def _cut(words: np.ndarray, wts: np.ndarray, k: int) -> List[List[int]]:
        """k - 1 increasing boundary keys at weighted quantiles (duplicates
        dropped: one key cannot be split)."""
        order = _lex_order(words)
        w = np.asarray(wts, np.float64)[order]
        cum = np.cumsum(w)
        out: List[List[int]] = []
        for j in range(1, k):
            i = int(np.searchsorted(cum, cum[-1] * j / k, side="right"))
            if i <= 0 or i >= len(order):
                continue
            b = [int(x) for x in words[:, order[i]]]
            if not out or b > out[-1]:
                out.append(b)
        return out

    def imbalance(self) -> float:
        """max / mean of the ranks' assigned work."""
        return max(self.load) / max(float(np.mean(self.load)), 1e-30)

    def _piece_mask(self, words: np.ndarray, lo, hi, upper_words=None) -> np.ndarray:
        """Columns of words [W][n] inside [lo, hi); with upper_words the
        columns are ranges [words, upper_words] overlapping it."""
        up = words if upper_words is None else upper_words
        m = np.ones(words.shape[1], bool)
        if lo is not None:
            m &= _geq(up, lo)
        if hi is not None:
            m &= ~_geq(words, hi)
        return m

    def row_mask(self, gid: np.ndarray, words: np.ndarray, rank: int) -> np.ndarray:
        """Window rows (gid [n], key words [W][n]) this rank holds."""
        gid = np.asarray(gid, np.int64)
        mine = [g for g, r in self.owner.items() if r == rank]
        m = np.isin(gid, mine)
        for g, parts in self.split.items():
            sel = np.nonzero(gid == g)[0]
            for lo, hi, r in parts:
                if r == rank and len(sel):
                    m[sel[self._piece_mask(words[:, sel], lo, hi)]] = True
        return m

    def range_mask(self, m: dict, rank: int) -> np.ndarray:
        lut = np.full(max(list(self.owner) + list(self.split) + [0]) + 1, -1, dtype=np.int64)
        for g, r in self.owner.items():
            lut[g] = r
        gid = np.asarray(m["gid"], dtype=np.int64)
        owner = np.where(gid < len(lut), lut[np.minimum(gid, len(lut) - 1)], 0)
        out = owner == rank
        for g, parts in self.split.items():
            sel = np.nonzero(gid == g)[0]
            if not len(sel):
                continue
            lo_w, hi_w = m["lo"][:, sel], m["hi"][:, sel]
            for lo, hi, r in parts:
                if r == rank:
                    out[sel[self._piece_mask(lo_w, lo, hi, upper_words=hi_w)]] = True
        return out

    def lock_mask(self, m: dict, rank: int) -> np.ndarray:
        return np.full(m["n_lock"], rank == 0, dtype=bool)


def plan_groups(rows: np.ndarray, ranges: Optional[np.ndarray], world: int,
                keys_of: Callable[[int], Tuple[np.ndarray, np.ndarray]]) -> "GroupShards":
    """GroupShards over per-group row and range counts (work ROW_COST x rows
    + RANGE_COST x ranges); keys_of(g) -> (key words [W][n], weights [n]) is
    asked only for the groups heavier than total / (2 world), the ones the
    plan cuts."""
    rows = np.asarray(rows, np.float64)
    rng = np.zeros(len(rows)) if ranges is None else np.asarray(ranges, np.float64)
    n = max(len(rows), len(rng))
    work = ROW_COST * np.pad(rows, (0, n - len(rows))) + RANGE_COST * np.pad(rng, (0, n - len(rng)))
    load = {g: float(work[g]) for g in range(n) if work[g] > 0}
    cap = work.sum() / (2 * max(world, 1))
    split = {int(g): keys_of(int(g)) for g in np.nonzero(work > cap)[0]} if world > 1 else {}
    return GroupShards(load, world, split)


def group_work(gid: np.ndarray, words: np.ndarray, m: Optional[dict], world: int):
    """GroupShards inputs from window rows (gid [n], key words [W][n]) and a
    marshalled batch m (its range probes; None = rows only): per-group work
    ROW_COST x rows + RANGE_COST x ranges, and for the groups heavier than
    total / (2 world) the keys to cut them at (rows and range lower bounds,
    weighted the same way)."""
    gid = np.asarray(gid, np.int64)
    mg = None if m is None else np.asarray(m["gid"], np.int64)
    ng = int(max(gid.max(initial=-1), -1 if mg is None else mg.max(initial=-1))) + 1
    rows = np.bincount(gid, minlength=ng)
    rng = None if mg is None else np.bincount(mg, minlength=ng)

    def keys_of(g):
        rw = words[:, gid == g]
        parts, wts = [rw], [np.full(rw.shape[1], ROW_COST)]
        if m is not None:
            lo = m["lo"][:, mg == g]
            parts.append(lo)
            wts.append(np.full(lo.shape[1], RANGE_COST))
        return np.concatenate(parts, axis=1), np.concatenate(wts)
    gs = plan_groups(rows, rng, world, keys_of)
    return gs


# ---- configs 2 / 5: sampled global splitters ---------------------------------
# A skewed key law (config 5: one Zipf(1.2) over 2^32 keys, hot keys at the low
# end) defeats fixed spans: nearly every distinct key and every hot range falls
# into one span.  The splitters are instead quantiles of the probe phase's
# work over the key space, estimated from a sample every rank contributes
# (one all_gather at window build): each rank's distinct window keys (after
# its local dedupe; hot keys collapse there) weighted ROW_COST per row, and
# a strided share of the batch's range lower bounds weighted RANGE_COST per
# range (measured per-unit probe time; SURVEY.md §8(d)'s byte model
# N_w s_w + N_r s_r underweights ranges, whose records are written and read
# back by the scatter and the join).  Rows then move to their
# owners with one all_to_all (exchange_rows); ranges that straddle a
# splitter go to both sides (KeyRangeShards routing).

INT64_MIN, INT64_MAX = -(1 << 63), (1 << 63) - 1
# Relative probe-phase cost of one distinct window row and one routed range on
# the narrow tile pipeline, fitted to a 2-rank config-5 run on MI355X
# (t = a rows + b ranges: a ~ 17 ps, b ~ 54 ps; profiles/r02_c5_gloo2.log).
ROW_COST, RANGE_COST = 1.0, 3.0


def sampled_splitters(local_keys: np.ndarray, range_keys: np.ndarray, world: int, rank: int,
                      w_row: float, w_range: float, samples: int = 4096, group=None) -> dict:
    """world - 1 int64 splitters (rank j owns key values [split[j-1], split[j]))
    balancing w_row * distinct window rows + w_range * ranges, identical on
    every rank.  local_keys: this rank's window key values (any order,
    duplicates allowed); range_keys: lower key values of the (global) batch's
    ranges.  Returns dict(splitters int64[world-1], and the sample's estimate
    of the per-rank load under these splitters and under fixed spans of
    [0, 2^key_bits) for comparison, in the caller's units)."""
    import torch
    import torch.distributed as dist
    uk, cnt = np.unique(np.asarray(local_keys, np.int64), return_counts=True)
    rk = np.sort(np.asarray(range_keys, np.int64)[rank::world])
    s_w = min(samples, len(uk))
    s_r = min(samples, len(rk))
    # evenly spaced order statistics of the distinct keys; each stands for the
    # keys up to the next one.  A key this rank wrote more than once is hot:
    # every rank almost surely holds it too, and it is one row after the
    # exchange -- so it counts 1 / world here (the tail's keys count 1).
    iw = (np.arange(s_w) * len(uk)) // max(s_w, 1)
    cum = np.concatenate([[0.0], np.cumsum(np.where(cnt >= 2, 1.0 / world, 1.0))])
    row_w = w_row * (cum[np.append(iw[1:], len(uk))] - cum[iw]) if s_w else np.zeros(0)
    ir = (np.arange(s_r) * len(rk)) // max(s_r, 1)
    keys = np.concatenate([uk[iw], rk[ir]])
    wts = np.concatenate([row_w, np.full(s_r, w_range * len(rk) / max(s_r, 1))])
    if dist.is_initialized():  # world 1 with a process group: a one-rank gather (RCCL smoke)
        n = 2 * samples
        kb = torch.full((n,), INT64_MAX, dtype=torch.int64)
        wb = torch.zeros(n, dtype=torch.float64)
        kb[:len(keys)] = torch.from_numpy(keys)
        wb[:len(wts)] = torch.from_numpy(wts)
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if dist.get_backend(group) == "nccl" else torch.device("cpu")
        kb, wb = kb.to(dev), wb.to(dev)
        ks = [torch.empty_like(kb) for _ in range(world)]
        ws = [torch.empty_like(wb) for _ in range(world)]
        dist.all_gather(ks, kb, group=group)
        dist.all_gather(ws, wb, group=group)
        keys = torch.cat(ks).cpu().numpy()
        wts = torch.cat(ws).cpu().numpy()
    order = np.argsort(keys, kind="stable")
    keys, wts = keys[order], wts[order]
    cum = np.cumsum(wts)
    total = cum[-1] if len(cum) else 0.0
    split = []
    for j in range(1, world):
        i = int(np.searchsorted(cum, total * j / world, side="left"))
        k = int(keys[min(i, len(keys) - 1)]) if len(keys) else 0
        if split and k <= split[-1]:
            k = split[-1] + 1  # a single hot key cannot be split: keep splitters increasing
        split.append(k)
    split = np.asarray(split, np.int64)

    def load(bounds):
        own = np.searchsorted(bounds, keys, side="right")
        return np.bincount(own, weights=wts, minlength=world)[:world]
    return dict(splitters=split, est_load=load(split), load=load)


def exchange_rows(keys: np.ndarray, lsn: np.ndarray, splitters: np.ndarray, group=None):
    """Move window rows (int64 key values, u64 commit LSNs) to the rank owning
    their key (one all_to_all; on RCCL through device buffers).  Returns this
    rank's (keys, lsn)."""
    import torch
    import torch.distributed as dist
    world = len(splitters) + 1
    if not dist.is_initialized():
        return keys, lsn
    own = np.searchsorted(splitters, keys, side="right")
    order = np.argsort(own, kind="stable")
    cnt = np.bincount(own, minlength=world).astype(np.int64)
    dev = torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend(group) == "nccl" else torch.device("cpu")
    send_n = torch.from_numpy(cnt).to(dev)
    recv_n = torch.empty_like(send_n)
    dist.all_to_all_single(recv_n, send_n, group=group)
    rc = recv_n.cpu().numpy().tolist()
    sc = cnt.tolist()
    out = []
    for a in (np.asarray(keys, np.int64), np.asarray(lsn, np.uint64).view(np.int64)):
        src = torch.from_numpy(np.ascontiguousarray(a[order])).to(dev)
        dst = torch.empty(int(sum(rc)), dtype=torch.int64, device=dev)
        dist.all_to_all_single(dst, src, output_split_sizes=rc, input_split_sizes=sc, group=group)
        out.append(dst.cpu().numpy())
    return out[0], out[1].view(np.uint64)


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


def gather_bitmaps(bitmap, gathered, group=None) -> None:
    """gathered[k * words ...] := rank k's verdict bitmap (one all-gather of
    n_txn / 8 bytes per rank; RCCL has no bitwise-OR reduction, so the ranks
    OR the N bitmaps themselves: hsc_or_bitmaps).  Per rank a ring all-gather
    moves (N - 1) n_txn / 8 bytes, a byte-wise max all-reduce 2 (N - 1) / N
    n_txn."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(gathered, bitmap, group=group)
    else:
        dist.all_gather(list(gathered.view(world, -1).unbind(0)), bitmap, group=group)


# ---- the C multi-GPU context (hsc_multi_*): composite splitters -------------
# The native multi context cuts the window into contiguous pieces of the
# composite key space (gid, key words); a piece boundary may fall inside a
# group (a hot group is cut) or between groups.  These helpers compute such
# splitters from rows (and optionally range lower bounds, weighted by their
# probe cost) and the owner of each row, with the C routing rule
# owner(K) = #splitters <= K.

def _composite_ge(gid, words, g, w):
    """rows (gid [n], words [W][n]) >= the composite key (g, w[W])."""
    gid = np.asarray(gid, np.int64)
    return (gid > int(g)) | ((gid == int(g)) & _geq(words, [int(x) for x in w]))


def composite_owner(gid, words, sp_gid, sp_w) -> np.ndarray:
    """Owner of every row: the number of splitters <= its composite key."""
    own = np.zeros(len(gid), np.int64)
    for k in range(len(sp_gid)):
        own += _composite_ge(gid, words, sp_gid[k], sp_w[:, k])
    return own


def composite_splitters(gid, words, world: int, m: Optional[dict] = None):
    """world - 1 ascending composite splitters (gid u32[S], words u64[W][S]) at
    equal-work quantiles of the rows (ROW_COST each) and, with a marshalled
    batch m, its range lower bounds (RANGE_COST each)."""
    gid = np.asarray(gid, np.int64)
    W = words.shape[0]
    g_all, w_all, wt = [gid], [words], [np.full(len(gid), ROW_COST)]
    if m is not None and m["n"]:
        g_all.append(np.asarray(m["gid"], np.int64))
        w_all.append(np.asarray(m["lo"], np.uint64)[:W])
        wt.append(np.full(m["n"], RANGE_COST))
    g = np.concatenate(g_all)
    w = np.concatenate(w_all, axis=1)
    wt = np.concatenate(wt)
    order = np.lexsort(tuple(w[::-1]) + (g,)) if len(g) else np.zeros(0, np.int64)
    cum = np.cumsum(wt[order])
    sp_g = np.zeros(world - 1, np.uint32)
    sp_w = np.zeros((W, world - 1), np.uint64)
    for j in range(1, world):
        i = int(np.searchsorted(cum, cum[-1] * j / world, side="left")) if len(cum) else 0
        i = min(i, len(order) - 1)
        if i >= 0 and len(order):
            sp_g[j - 1] = g[order[i]]
            sp_w[:, j - 1] = w[:, order[i]]
    return sp_g, sp_w


def int64_splitter_keys(splitters, W: int):
    """int64 key-value splitters (rank j owns [s[j-1], s[j])) as composite
    splitters of group 0 (9-byte memcmp keys, formats.enc_int64)."""
    sp = [int(x) for x in splitters]
    sp_g = np.zeros(len(sp), np.uint32)
    sp_w = np.zeros((W, len(sp)), np.uint64)
    for k, v in enumerate(sp):
        sp_w[:, k] = key_words(F.enc_int64(v), W)
    return sp_g, sp_w


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
