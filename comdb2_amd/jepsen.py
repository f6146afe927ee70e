"""Jepsen-format histories -> dependency-graph histories.

The reference's Jepsen harness records operation histories as EDN, one map
per line, an ``:invoke`` and its completion (``:ok`` / ``:fail`` / ``:info``)
per process:

* the C register client (linearizable/ctest/register.c:282-370): one
  register (``id = 1``), ``:f :read`` (completes with the observed ``:value``
  and ``:uid``, ``nil`` for an empty register), ``:f :write :value v :uid u``
  and ``:f :cas :value [cur new] :uid u`` (``update ... where val = cur``);
  every txn runs SERIALIZABLE (register.c:270);
* Adya's G2 workload (linearizable/jepsen/src/jepsen/adya.clj:13-55):
  ``:f :insert :value [key [a-id b-id]]`` -- the txn reads tables a and b for
  the key and inserts its row into one of them only if both were empty; the
  G2 checker (:57-83) flags a key with more than one ``:ok`` insert.

:func:`history_from_jepsen_edn` pairs each invoke with its completion (a
history may also be one EDN vector of ops, as knossos reads it:
linearizable/filetest/src/jepsen/filetest.clj, ``history.txt``), drops
``:fail`` ops (not committed), and turns every ``:ok`` op into one committed
transaction of a :class:`workloads.History`:

* txn ids = commit order, taken as the order of the completions (their
  ``:time``, else their line order); a key's version order is its writers'
  txn order;
* register read: a read of the version it returned -- the writer with the
  same ``:uid`` and value when the op carries a ``:uid`` (register.c), else
  the writer of the same value (a knossos register history of unique
  values); the latest such writer before it, else the earliest after it;
  ``nil`` = the initial, empty register;
* register write: a write of the register;
* register cas ``[cur new]``: a read of the latest earlier version whose value
  is ``cur`` (the version the ``where val = cur`` matched: the CAS chain)
  plus a write;
* insert ``[k [a b]]``: reads of ``(k, a)`` and ``(k, b)`` that saw the
  initial (absent) rows, plus a write of ``(k, a)`` or ``(k, b)``.

``:info`` ops are indeterminate: they may have committed.  Their writes stay
candidate versions, and one that a read observed (no ``:ok`` writer produced
that version) did commit -- it joins the history as a transaction ordered at
its invoke (``info_recovered``); the others are dropped.  Reads whose version
no writer produced are dropped and counted (``dangling``).  hsc_dep_graph_*
then builds the WR / WW / RW edges and the SCCs; a nontrivial SCC is a
dependency cycle (two ``:ok`` inserts of one G2 key form the 2-cycle of rw
edges the G2 checker looks for).
"""
from __future__ import annotations

import dataclasses
import re
from typing import Dict, List, Optional, Tuple

import numpy as np

from .workloads import History

# ---------------------------------------------------------------------------
# EDN (the subset the histories use: maps, vectors, keywords, integers, nil,
# booleans, strings)
# ---------------------------------------------------------------------------
_TOK = re.compile(r'\s*(?:,\s*)*([{}\[\]()]|"(?:[^"\\]|\\.)*"|[^\s,{}\[\]()"]+)')


def _tokens(text: str):
    pos = 0
    while True:
        m = _TOK.match(text, pos)
        if not m or m.end() == pos:
            return
        pos = m.end()
        yield m.group(1)


def _parse(tokens, tok):
    if tok in ("{", "[", "("):
        close = {"{": "}", "[": "]", "(": ")"}[tok]
        items = []
        for t in tokens:
            if t == close:
                break
            items.append(_parse(tokens, t))
        else:
            raise ValueError("unterminated EDN collection")
        if tok == "{":
            if len(items) % 2:
                raise ValueError("odd EDN map")
            return dict(zip(items[::2], items[1::2]))
        return items
    if tok in ("}", "]", ")"):
        raise ValueError(f"unexpected {tok!r}")
    if tok == "nil":
        return None
    if tok in ("true", "false"):
        return tok == "true"
    if tok.startswith('"'):
        return tok[1:-1]
    if re.fullmatch(r"[-+]?\d+N?", tok):
        return int(tok.rstrip("N"))
    return tok  # keywords stay strings (":ok")


def parse_edn(text: str) -> List:
    """Every top-level EDN form of text, in order."""
    toks = _tokens(text)
    return [_parse(toks, t) for t in toks]


# ---------------------------------------------------------------------------
# history -> dependency-graph ops
# ---------------------------------------------------------------------------
@dataclasses.dataclass
class JepsenOps:
    """What the conversion kept and dropped."""
    history: History
    ok: int                  # completed :ok ops (committed txns)
    failed: int              # :fail completions (dropped)
    info: int                # :info completions (indeterminate)
    unpaired: int            # invokes without a completion
    dangling: int            # reads of a version no writer produced (dropped)
    g2_keys: Dict[int, int]  # insert key -> :ok inserts (adya.clj g2-checker input)
    txn_ops: List[dict]      # the completion of each txn (txn id order)
    info_recovered: int = 0  # :info ops whose write a read observed (committed)


def _flatten(forms):
    for f in forms:
        if isinstance(f, list):  # a history vector [op op ...]
            yield from _flatten(f)
        else:
            yield f


def _pairs(forms):
    """(ok, info, failed, unpaired): ok / info = [(invoke, completion, line)]."""
    pending: Dict[object, Tuple[dict, int]] = {}
    done, infos, failed = [], [], 0
    for i, op in enumerate(_flatten(forms)):
        if not isinstance(op, dict):
            continue
        t, p = op.get(":type"), op.get(":process")
        if t == ":invoke":
            pending[p] = (op, i)
        elif t in (":ok", ":fail", ":info"):
            inv = pending.pop(p, (None, -1))[0]
            if t == ":fail":
                failed += 1
            elif t == ":info":
                infos.append((inv or {}, op, i))
            else:
                done.append((inv or {}, op, i))
    return done, infos, failed, len(pending)


_INSERT_TABLES = 2  # adya.clj: tables a and b


def _time(op, line):
    t = op.get(":time")
    return t if isinstance(t, int) else line


def history_from_jepsen_edn(text: str) -> JepsenOps:
    """See the module docstring.  Register keys are ``:key`` when an op
    carries one (the reference's client has a single register, id 1); G2
    insert keys become (key, table) = 2 key + {0: a, 1: b}."""
    done, infos, failed, unpaired = _pairs(parse_edn(text))
    # every op that may be a txn: (order time, line, invoke, completion, is :ok)
    # -- an :ok op commits at its completion, an :info op (if at all) by its
    # completion, taken as its invoke
    cands = [(_time(op, i), i, inv, op, True) for inv, op, i in done]
    cands += [(_time(inv, i) if inv else i, i, inv, op, False) for inv, op, i in infos
              if op.get(":f", inv.get(":f")) in (":write", ":cas")]
    cands.sort(key=lambda c: (c[0], c[1]))
    # per candidate: its ops as (key, is_write, read kind, a, b)
    ops_of: List[List[tuple]] = []
    writers: Dict[int, List[Tuple[int, object, object]]] = {}  # key -> [(cand, uid, value)]
    g2: Dict[int, int] = {}
    for c, (_, _, inv, op, ok) in enumerate(cands):
        f = op.get(":f", inv.get(":f"))
        mine = []
        if f in (":read", ":write", ":cas"):
            k = int(op.get(":key", inv.get(":key", 1)))
            if f == ":read":
                if ":uid" in op:
                    mine.append((k, 0, "uid", op.get(":uid"), op.get(":value")))
                else:
                    mine.append((k, 0, "value", op.get(":value"), None))
            else:
                val = op.get(":value", inv.get(":value"))
                if f == ":cas":
                    cur, val = val
                    mine.append((k, 0, "cas", cur, None))
                writers.setdefault(k, []).append((c, op.get(":uid", inv.get(":uid")), val))
                mine.append((k, 1, None, None, None))
        elif f == ":insert":
            k, (a_id, b_id) = op.get(":value", inv.get(":value"))
            g2[int(k)] = g2.get(int(k), 0) + 1
            for tb in range(_INSERT_TABLES):  # both tables read empty
                mine.append((2 * int(k) + tb, 0, "none", None, None))
            mine.append((2 * int(k) + (0 if a_id is not None else 1), 1, None, None, None))
        ops_of.append(mine)

    def observed(c, k, kind, a, b):
        """The candidate whose version a read of candidate c saw (None:
        initial; -1: no writer produced it)."""
        if kind == "none" or (kind in ("uid", "value") and a is None):
            return None
        ws = writers.get(k, [])
        if kind == "cas":
            hits = [w for w, u, v in reversed(ws) if w < c and v == a]
            hits = [w for w in hits if cands[w][4]] or hits  # :ok writers first
            return hits[0] if hits else -1
        if kind == "uid":
            match = [w for w, u, v in ws if u == a and (b is None or v == b)]
        else:
            match = [w for w, u, v in ws if v == a]
        for pool in ([w for w in match if cands[w][4]], match):  # :ok writers first
            before = [w for w in pool if w < c]
            if before:
                return before[-1]
            if pool:
                return pool[0]
        return -1

    keep = [c[4] for c in cands]  # :ok ops; observed :info writes join below
    seen: Dict[Tuple[int, int], object] = {}
    for c, mine in enumerate(ops_of):
        if not cands[c][4]:
            continue
        for j, (k, w, kind, a, b) in enumerate(mine):
            if not w:
                seen[(c, j)] = observed(c, k, kind, a, b)
    # an :info write a committed read observed did commit (and its own reads
    # then count too)
    changed = True
    while changed:
        changed = False
        for (c, j), hit in list(seen.items()):
            if isinstance(hit, int) and hit >= 0 and not keep[hit]:
                keep[hit] = True
                changed = True
                for jj, (k, w, kind, a, b) in enumerate(ops_of[hit]):
                    if not w:
                        seen[(hit, jj)] = observed(hit, k, kind, a, b)
    tid = {}
    for c in range(len(cands)):
        if keep[c]:
            tid[c] = len(tid)
    txn, key, isw, obs = [], [], [], []
    dangling = 0
    for c, mine in enumerate(ops_of):
        if not keep[c]:
            continue
        for j, (k, w, kind, a, b) in enumerate(mine):
            o = -1
            if not w:
                hit = seen.get((c, j))
                if hit is not None and (hit < 0 or not keep[hit]):
                    dangling += 1
                    continue
                o = -1 if hit is None else tid[hit]
            txn.append(tid[c]), key.append(k), isw.append(w), obs.append(o)
    h = History(np.array(txn, np.uint32), np.array(key, np.uint64), np.array(isw, np.uint8),
                np.array(obs, np.int64), len(tid))
    recovered = sum(1 for c in range(len(cands)) if keep[c] and not cands[c][4])
    return JepsenOps(h, len(done), failed, len(infos), unpaired, dangling, g2,
                     [cands[c][3] for c in range(len(cands)) if keep[c]], recovered)


def g2_illegal(ops: JepsenOps) -> Dict[int, int]:
    """adya.clj g2-checker (:57-83): the insert keys with more than one :ok
    insert."""
    return {k: c for k, c in ops.g2_keys.items() if c > 1}


# ---------------------------------------------------------------------------
# generated histories (test inputs; the reference's clients need a live
# cluster and a JVM)
# ---------------------------------------------------------------------------
def register_history_edn(seed: int, n_ops: int = 2000, n_procs: int = 8, n_keys: int = 1,
                         lost_update: float = 0.02, stale_read: float = 0.05,
                         fail: float = 0.05) -> Tuple[str, int]:
    """A register.c-shaped history (read / write / cas, values rand() % 5,
    uids rand() % 100000) of a serial execution with injected anomalies:
    ``lost_update`` -- a cas whose ``cur`` is the value of an older version
    than the latest (both 'saw' it: a cycle with the writer in between);
    ``stale_read`` -- a read returning an older version.  Completions are
    logged in commit order, each op's invoke at a random earlier time (ops
    of one process never overlap).  n_keys > 1 adds ``:key`` (independent
    registers).  Returns (EDN text, injected lost updates)."""
    rng = np.random.default_rng(seed)
    versions: Dict[int, List[Tuple[int, int]]] = {k: [] for k in range(1, n_keys + 1)}
    lines: List[Tuple[int, int, str]] = []
    busy = np.zeros(n_procs, np.int64)
    now, lost = 1000, 0
    for _ in range(n_ops):
        now += int(rng.integers(1, 50))
        p = int(rng.integers(0, n_procs))
        inv_t = max(int(busy[p]) + 1, now - int(rng.integers(0, 400)))
        k = int(rng.integers(1, n_keys + 1))
        kk = f" :key {k}" if n_keys > 1 else ""
        vs = versions[k]
        op = int(rng.integers(0, 3))
        uid = int(rng.integers(0, 100000))
        new = int(rng.integers(0, 5))
        ok = rng.random() >= fail
        if op == 0:
            inv = f"{{:type :invoke :f :read :value nil :process {p}{kk} :time {inv_t}}}"
            if vs and rng.random() < stale_read and len(vs) > 1:
                v, u = vs[int(rng.integers(0, len(vs) - 1))]
            else:
                v, u = vs[-1] if vs else (None, None)
            body = (f":f :read :process {p} :value {'nil' if v is None else v} "
                    f":uid {'nil' if u is None else u}")
        elif op == 1:
            inv = f"{{:type :invoke :f :write :value {new} :process {p}{kk} :uid {uid} :time {inv_t}}}"
            body = f":f :write :process {p} :value {new} :uid {uid}"
            if ok:
                vs.append((new, uid))
        else:
            if vs and len(vs) > 1 and rng.random() < lost_update and vs[-2][0] != vs[-1][0]:
                cur = vs[-2][0]  # matched an older version: a lost update
                lost += ok
            elif vs:
                cur = vs[-1][0]
            else:
                cur, ok = int(rng.integers(0, 5)), False  # empty register: the update hits no row
            inv = (f"{{:type :invoke :f :cas :value [{cur} {new}] :process {p}{kk} :uid {uid} "
                   f":time {inv_t}}}")
            body = f":f :cas :process {p} :value [{cur} {new}] :uid {uid}"
            if ok:
                vs.append((new, uid))
        kind = ":ok" if ok else ":fail"
        lines.append((inv_t, len(lines), inv))
        lines.append((now, len(lines), f"{{:type {kind} {body}{kk} :time {now}}}"))
        busy[p] = now
    lines.sort()
    return "\n".join(l for _, _, l in lines) + "\n", lost


def adya_g2_edn(seed: int, n_keys: int = 500, anomaly: float = 0.05) -> Tuple[str, List[int]]:
    """adya.clj g2-gen's history (two concurrent inserts per key, one with an
    a-id and one with a b-id, globally unique ids): normally the first
    committer succeeds and the other fails serialization; with probability
    ``anomaly`` both complete :ok (G2).  Returns (EDN text, anomalous keys)."""
    rng = np.random.default_rng(seed)
    ids, t, lines, bad = 0, 1000, [], []
    for k in range(n_keys):
        pa, pb = 2 * (k % 8), 2 * (k % 8) + 1
        ids += 2
        a, b = ids - 1, ids
        both = rng.random() < anomaly
        first = int(rng.integers(0, 2))
        t0 = t
        lines.append(f"{{:type :invoke :f :insert :value [{k} [{a} nil]] :process {pa} :time {t0}}}")
        lines.append(f"{{:type :invoke :f :insert :value [{k} [nil {b}]] :process {pb} :time {t0 + 1}}}")
        for j, (p, val) in enumerate(((pa, f"[{k} [{a} nil]]"), (pb, f"[{k} [nil {b}]]"))):
            ok = both or j == first
            lines.append(f"{{:type {':ok' if ok else ':fail'} :f :insert :value {val} "
                         f":process {p} :time {t0 + 2 + j}}}")
        if both:
            bad.append(k)
        t += 10
    return "\n".join(lines) + "\n", bad
