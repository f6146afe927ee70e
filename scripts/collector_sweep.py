"""Collector throughput / latency against the in-flight bound (GPU box):
64 (and 32, 128) native caller threads over a config-2 window, each setting
run 3 times (the spread between runs is of the order of the differences)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from comdb2_amd.hsc import NativeCurRangeArrs, Validator  # noqa: E402
from comdb2_amd.workloads import config2, config2_device_window  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

v = Validator(0)
assert v.register_group("t1", 0, 9) == 0
wl = config2(n_commits=1_000_000, n_txn=20_000, seed=5, build_log=False)
gid, words, lsn = config2_device_window(wl)
dev = torch.device("cuda:0")
tg = torch.from_numpy(gid).to(dev)
tw = torch.from_numpy(words.reshape(-1).view(np.int64)).to(dev)
tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
v.ingest_device(len(lsn), words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(),
                wl.params["end_lsn"])
torch.cuda.synchronize()
arrs = NativeCurRangeArrs(wl.readsets)
for threads in (32, 64, 128):
    for inflight in (1, 2, 3, 4):
        for rep in range(3):
            _, st = v.concurrent_check(arrs, nthreads=threads, inflight=inflight)
            keep = {k: (round(x, 1) if isinstance(x, float) else x) for k, x in st.items()
                    if k in ("checks_per_s", "lat_p50_us", "lat_p99_us", "mean_batch",
                             "device_pass_us", "gate_us", "handout_us")}
            print(json.dumps({"threads": threads, "inflight": inflight, "rep": rep, **keep}), flush=True)
arrs.close()
v.close()
