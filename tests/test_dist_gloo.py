"""CPU, world sizes 2, 4 and 8 over gloo: the sharded check
(comdb2_amd/shard.py) -- marshal the global batch, route probes to key-range
/ group shards, evaluate each shard's probes against only that shard's
window, merge verdict bytes with all_reduce(MAX) -- must equal the unsharded
oracle verdicts; configs 3 and 5 also report and bound the per-rank work
imbalance (max / mean)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _merge_logs(logs):
    from comdb2_amd.formats import LLog
    keys, offs = [], []
    base = 0
    for lg in logs:
        keys.append(lg.keys)
        offs.append(lg.key_off + np.uint64(base))
        base += len(lg.keys)
    cat = lambda name: np.concatenate([getattr(lg, name) for lg in logs])
    lsn = cat("lsn")
    order = np.argsort(lsn, kind="stable")
    pick = lambda a: a[order]
    return LLog(pick(lsn), pick(cat("rectype")), pick(cat("prev")), pick(cat("isabort")),
                pick(cat("table")), pick(cat("ix")), pick(np.concatenate(offs)),
                pick(cat("keylen")), np.concatenate(keys), logs[0].tbnames,
                max(int(lg.end_lsn) for lg in logs))


def _worker(rank, world, port, mode, out_path):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist

    from comdb2_amd import shard
    from comdb2_amd.hsc import Validator
    from comdb2_amd.workloads import config2, random_case
    from probe_model import WindowModel, evaluate

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    v = Validator(-1)
    if mode in ("config5", "config3"):
        (_config5_rank if mode == "config5" else _config3_rank)(rank, world, v, out_path)
        dist.barrier()
        dist.destroy_process_group()
        v.close()
        return
    if mode == "keyrange":
        kw = dict(n_commits=1500, n_txn=300, value_bits=18, width=1 << 9, snap_recent=0.5)
        shards_logs = [config2(rank=r, world=world, **kw).log for r in range(world)]
        glog = _merge_logs(shards_logs)
        rs = config2(rank=rank, world=world, build_log=False, **kw).readsets
        v.ingest_log(glog)
        m = v.marshal(rs)
        sh = shard.KeyRangeShards.int64_uniform(world, kw["value_bits"], m["words"])
        local = WindowModel(shards_logs[rank])
    else:
        glog, rs = random_case(77, n_commits=120, n_txn=80)
        v.ingest_log(glog)
        m = v.marshal(rs)
        full = WindowModel(glog)
        sizes = {}
        gid = 0
        while True:
            try:
                tid, ix, kl = v.group_info(gid)
            except Exception:
                break
            sizes[gid] = len(full.groups.get((v.table_name(tid), ix, kl), ([], []))[0])
            gid += 1
        sh = shard.GroupShards(sizes, world)
        mine = {(v.table_name(v.group_info(g)[0]),) + v.group_info(g)[1:]
                for g, r in sh.owner.items() if r == rank}
        local = WindowModel(glog, key_filter=lambda tb, ix, key: (tb, ix, len(key)) in mine)
    # table maxima: each shard's own view, merged across ranks
    names = sorted(local.table_max)
    tm = np.array([local.table_max[n] for n in names], dtype=np.uint64)
    merged_tm = shard.allreduce_table_max(tm)
    sub = shard.route(m, sh.range_mask(m, rank), sh.lock_mask(m, rank))
    verdict = evaluate(v, sub, local, table_max_by_name=dict(zip(names, merged_tm.tolist())))
    # the bench's merge: all-gather of the shards' verdict bitmaps, OR-ed
    n = len(verdict)
    words = (n + 63) // 64
    bits = np.zeros(words * 8, np.uint8)
    bits[: (n + 7) // 8] = np.packbits(verdict != 0, bitorder="little")
    gathered = torch.zeros(world * words, dtype=torch.int64)
    shard.gather_bitmaps(torch.from_numpy(bits.view(np.int64).copy()), gathered)
    ored = np.bitwise_or.reduce(gathered.numpy().reshape(world, words), axis=0)
    by_bits = np.unpackbits(ored.view(np.uint8), bitorder="little")[:n]
    t = torch.from_numpy(verdict.copy())
    shard.merge_verdicts(t)
    assert np.array_equal(by_bits != 0, t.numpy() != 0)  # both merges agree
    if rank == 0:
        np.save(out_path, np.maximum(t.numpy(), m["forced"]))
    dist.barrier()
    dist.destroy_process_group()
    v.close()


C5_KW = dict(keys_per_gpu=20_000, n_txn=300, snap_recent=0.3)
W_ROW, W_RANGE = 1.0, 3.0  # shard.ROW_COST / RANGE_COST


def _config5_rank(rank, world, v, out_path):
    """Config 5 on `world` gloo ranks: rank r's segment of the global Zipf
    log, sampled global splitters, one all_to_all of the rows to their
    owners, the batch routed by the splitters, each shard's probes joined
    against its own rows (oracle/sortjoin.c, the CPU stand-in for the HIP
    join), verdicts merged with all_reduce(MAX)."""
    import json
    import time

    import torch
    import torch.distributed as dist

    from comdb2_amd import shard
    from comdb2_amd.workloads import config5_scaled, int64_words
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    c5 = config5_scaled(rank=rank, world=world, **C5_KW)
    sp = shard.sampled_splitters(c5.keys, c5.range_keys, world, rank, W_ROW, W_RANGE,
                                 samples=1024)
    keys, lsn = shard.exchange_rows(c5.keys, c5.lsn, sp["splitters"])
    v.register_group("t1", 0, 9)
    v.set_end(c5.end_lsn)
    m = v.marshal(c5.readsets)
    sh = shard.KeyRangeShards.int64_splitters(sp["splitters"], m["words"])
    sub = shard.route(m, sh.range_mask(m, rank), sh.lock_mask(m, rank))
    tmax = shard.allreduce_table_max(np.array([lsn.max() if len(lsn) else 0], np.uint64))
    sj = oracle.SortJoin(np.zeros(len(keys), np.uint32), int64_words(keys), lsn, 1)
    t0 = time.perf_counter()
    verdict, _ = sj.probe(sub, tmax, nthreads=1)
    secs = time.perf_counter() - t0
    rows = sj.rows
    sj.close()
    t = torch.from_numpy(verdict.copy())
    shard.merge_verdicts(t)
    loc = torch.tensor([rows, sub["n"], secs], dtype=torch.float64)
    allg = [torch.zeros_like(loc) for _ in range(world)]
    dist.all_gather(allg, loc)
    per = torch.stack(allg).numpy()
    fixed = np.array([(j << 32) // world for j in range(1, world)], np.int64)
    if rank == 0:
        np.save(out_path, t.numpy())
        work = per[:, 0] * W_ROW + per[:, 1] * W_RANGE
        est_fixed = sp["load"](fixed)
        with open(out_path + ".json", "w") as f:
            json.dump({"splitters": sp["splitters"].tolist(), "rows_per_rank": per[:, 0].tolist(),
                       "ranges_per_rank": per[:, 1].tolist(),
                       "probe_s_per_rank": per[:, 2].tolist(),
                       "time_max_over_mean": float(per[:, 2].max() / per[:, 2].mean()),
                       "work_max_over_mean": float(work.max() / work.mean()),
                       "est_max_over_mean": float(sp["est_load"].max() / sp["est_load"].mean()),
                       "fixed_span_est_max_over_mean": float(est_fixed.max() / est_fixed.mean())},
                      f)


C3_KW = dict(n_writes=120_000, n_txn=600)


def _config3_rank(rank, world, v, out_path):
    """Config 3 over `world` ranks: every rank builds the same plan
    (shard.group_work + GroupShards: LPT over groups by rows + 3 x ranges,
    hot groups cut into key-range pieces), keeps the rows of its pieces,
    probes the ranges routed to them (oracle/sortjoin.c, the CPU stand-in for
    the HIP join) and the verdicts are merged with all_reduce(MAX)."""
    import json

    import torch
    import torch.distributed as dist

    from comdb2_amd import shard
    from comdb2_amd.workloads import config3_arrays
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    a = config3_arrays(**C3_KW)
    gid, words, lsn = a.window()
    for g, (tb, ix, L) in enumerate(a.groups):
        assert v.register_group(tb, ix, L) == g
    v.set_end(a.end_lsn)
    m = v.marshal(a.readsets)
    gs = shard.group_work(gid, words, m, world)
    sel = gs.row_mask(gid, words, rank)
    sub = shard.route(m, gs.range_mask(m, rank), gs.lock_mask(m, rank))
    sj = oracle.SortJoin(gid[sel], np.ascontiguousarray(words[:, sel]), lsn[sel], len(a.groups))
    verdict, _ = sj.probe(sub, a.table_max, nthreads=1)
    sj.close()
    t = torch.from_numpy(verdict.copy())
    shard.merge_verdicts(t)
    loc = torch.tensor([float(sel.sum()), float(sub["n"])], dtype=torch.float64)
    allg = [torch.zeros_like(loc) for _ in range(world)]
    dist.all_gather(allg, loc)
    per = torch.stack(allg).numpy()
    if rank == 0:
        np.save(out_path, t.numpy())
        work = per[:, 0] * shard.ROW_COST + per[:, 1] * shard.RANGE_COST
        with open(out_path + ".json", "w") as f:
            json.dump({"plan_max_over_mean": gs.imbalance(), "split_groups": sorted(gs.split),
                       "rows_per_rank": per[:, 0].tolist(), "ranges_per_rank": per[:, 1].tolist(),
                       "work_max_over_mean": float(work.max() / work.mean())}, f)


def _run(mode, tmp_path, world=2):
    import torch.multiprocessing as mp
    out = str(tmp_path / f"verdict_{mode}_{world}.npy")
    mp.start_processes(_worker, args=(world, _free_port(), mode, out), nprocs=world, join=True,
                       start_method="spawn")
    return np.load(out)


def test_keyrange_shards_match_oracle(tmp_path, oracle_mod):
    from comdb2_amd.workloads import config2
    got = _run("keyrange", tmp_path)
    kw = dict(n_commits=1500, n_txn=300, value_bits=18, width=1 << 9, snap_recent=0.5)
    logs = [config2(rank=r, world=2, **kw).log for r in range(2)]
    glog = _merge_logs(logs)
    rs = config2(rank=0, world=2, build_log=False, **kw).readsets
    want, _, _ = oracle_mod.check(glog, rs, nthreads=8)
    np.testing.assert_array_equal(got != 0, want != 0)
    assert 0 < int((want != 0).sum()) < len(want)


def test_group_shards_match_oracle(tmp_path, oracle_mod):
    from comdb2_amd.workloads import random_case
    got = _run("group", tmp_path)
    glog, rs = random_case(77, n_commits=120, n_txn=80)
    want, _, _ = oracle_mod.check(glog, rs)
    np.testing.assert_array_equal(got != 0, want != 0)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_config5_sampled_splitters_match_oracle(tmp_path, oracle_mod, world):
    """one global Zipf(1.2) over 2^32 keys; sampled global
    splitters balance the shards (a fixed split would not) and the merged
    verdicts equal the oracle's over the global log."""
    import json

    from comdb2_amd.workloads import config5_log, config5_scaled
    got = _run("config5", tmp_path, world)
    st = json.load(open(str(tmp_path / f"verdict_config5_{world}.npy") + ".json"))
    segs = [config5_scaled(rank=r, world=world, **C5_KW) for r in range(world)]
    glog = config5_log([s.keys for s in segs])
    want, _, _ = oracle_mod.check(glog, segs[0].readsets, nthreads=8)
    np.testing.assert_array_equal(got != 0, want != 0)
    assert 0 < int((want != 0).sum()) < len(want)
    assert st["fixed_span_est_max_over_mean"] > 1.25  # the skew is real (world = all on one rank)
    assert st["work_max_over_mean"] < 1.25            # and the splitters balance it
    assert "time_max_over_mean" in st


@pytest.mark.parametrize("world", [2, 4, 8])
def test_config3_split_group_shards_match_oracle(tmp_path, oracle_mod, world):
    """Config 3's (table, index) groups over 2 / 4 / 8 ranks: the merged
    verdicts equal the log oracle's, and the planned and the routed work stay
    balanced (max / mean <= 1.15) -- at 8 ranks only because the hot groups
    are cut into key-range pieces (whole groups by LPT: 1.7)."""
    import json

    from comdb2_amd import shard
    from comdb2_amd.workloads import config3_arrays, config3_log
    got = _run("config3", tmp_path, world)
    st = json.load(open(str(tmp_path / f"verdict_config3_{world}.npy") + ".json"))
    a = config3_arrays(**C3_KW)
    want, _, _ = oracle_mod.check(config3_log(a), a.readsets, nthreads=8)
    np.testing.assert_array_equal(got != 0, want != 0)
    assert 0 < int((want != 0).sum()) < len(want)
    assert st["plan_max_over_mean"] <= 1.15, st
    assert st["work_max_over_mean"] <= 1.15, st
    if world == 8:
        assert st["split_groups"], st
        gid, _, _ = a.window()
        whole = shard.GroupShards({g: float(n) for g, n in enumerate(np.bincount(gid))}, world)
        assert whole.imbalance() > 1.3  # without splitting


def test_config3_real_size_plan_balances_at_8():
    """The plan at config 3's bench size for 8 GPUs (8 x 4M index writes, the
    generator's group sizes; keys drawn only for the groups the plan cuts):
    LPT over whole groups is capped by the largest group (max / mean 1.72);
    with hot groups cut into key-range pieces it is <= 1.15."""
    from comdb2_amd import shard
    from comdb2_amd.workloads import SEED_CONFIG3, config3_group_keys, config3_group_sizes
    n_ix = 4
    sizes = config3_group_sizes(np.random.default_rng(SEED_CONFIG3), 8 * n_ix, 32_000_000)
    W = 8

    def keys_of(g):
        kb = config3_group_keys(SEED_CONFIG3, g, n_ix, int(sizes[g]), 1 << 12)
        pad = np.zeros((len(kb), 8 * W), np.uint8)
        pad[:, :kb.shape[1]] = kb
        words = pad.view(">u8").astype(np.uint64).reshape(len(kb), W).T
        return words, np.ones(len(kb))
    whole = shard.GroupShards({g: float(n) for g, n in enumerate(sizes)}, 8)
    split = shard.plan_groups(sizes, None, 8, keys_of)
    assert whole.imbalance() > 1.5
    assert split.imbalance() <= 1.15, split.imbalance()
    assert split.split
