"""rw conflict pairs before the OR-reduction (hsc_rw_edges)
on config 2 (10M logged int64 writes, 100k read sets x 10 ranges) without its
open-ended ranges (2 %: a range open on one side pairs with every later writer
of half the key space, hundreds of millions of pairs): GPU call time (marshal
+ upload + count/scan/emit + sort/dedupe + download) vs a vectorised numpy
restatement on the host (one core), checked equal."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from comdb2_amd import hsc
from comdb2_amd.workloads import config2, config2_device_window

c2 = config2(build_log=False)
gid, words, lsn = config2_device_window(c2)
v = hsc.Validator(0)
v.register_group("t1", 0, 9)
dev = torch.device("cuda", 0)
tg = torch.from_numpy(gid).to(dev); tw = torch.from_numpy(words.reshape(-1).view(np.int64)).to(dev)
tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
v.ingest_device(len(lsn), 2, tg.data_ptr(), tw.data_ptr(), tl.data_ptr(), c2.params["end_lsn"])
torch.cuda.synchronize()
import dataclasses
rs0 = c2.readsets
keep_r = (rs0.lflag == 0) & (rs0.rflag == 0)
cnt_t = np.add.reduceat(keep_r.astype(np.int64), rs0.txn_off[:-1]) if len(keep_r) else np.zeros(0, np.int64)
cnt_t[np.diff(rs0.txn_off) == 0] = 0
rs = dataclasses.replace(rs0, txn_off=np.concatenate([[0], np.cumsum(cnt_t)]).astype(np.int64),
                         **{f: getattr(rs0, f)[keep_r] for f in ("table", "idxnum", "lflag", "rflag",
                            "islocked", "lkeylen", "rkeylen", "lkey_off", "rkey_off")})
v.rw_edges(rs)  # warm
t0 = time.perf_counter(); txn, wl = v.rw_edges(rs); gpu = time.perf_counter() - t0

# numpy restatement: 9-byte int64 keys -> one u64 (drop the constant 0x08 byte)
t0 = time.perf_counter()
M = (1 << 56) - 1
def k64(w0, w1):
    top = w0 >> np.uint64(56)
    k = ((w0 & np.uint64(M)) << np.uint64(8)) | (w1 >> np.uint64(56))
    k = np.where(top < 8, np.uint64(0), k)
    return np.where(top > 8, np.uint64(np.iinfo(np.uint64).max), k)
kr = k64(words[0], words[1])
order = np.lexsort((lsn, kr))
kr, lr = kr[order], lsn[order]
m = v.marshal(rs)
klo, khi = k64(m["lo"][0], m["lo"][1]), k64(m["hi"][0], m["hi"][1])
a = np.searchsorted(kr, klo, "left"); b = np.maximum(a, np.searchsorted(kr, khi, "right"))
cnt = b - a
q = np.repeat(np.arange(m["n"]), cnt)
r = np.repeat(a, cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
keep = lr[r] > m["snap"][q]
pairs = np.unique((m["txn"][q[keep]].astype(np.uint64) << np.uint64(32)) | np.searchsorted(
    np.unique(lr), lr[r[keep]]).astype(np.uint64))
cpu = time.perf_counter() - t0
uc = np.unique(lr)
want_t = (pairs >> np.uint64(32)).astype(np.uint32); want_l = uc[(pairs & np.uint64(0xFFFFFFFF)).astype(np.int64)]
ok = np.array_equal(txn, want_t) and np.array_equal(wl, want_l)
n_r = m["n"]
print(json.dumps(dict(ranges=int(n_r), read_sets=rs.ntxn, pairs=int(len(txn)), gpu_s=gpu, cpu_numpy_s=cpu,
                      gpu_ranges_per_s=n_r / gpu, cpu_ranges_per_s=n_r / cpu, equal=bool(ok)), indent=1))
