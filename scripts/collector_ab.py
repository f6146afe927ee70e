"""Collector A/B on the GPU box: 64 native caller threads through the
collector over a config-2 window, 5 runs; the environment of this process
selects the variant (HSC_NO_PRE_ASSEMBLE, HSC_NO_STREAM_PRIO)."""
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
wl = config2(n_commits=1_000_000, n_txn=100_000, build_log=False)
gid, words, lsn = config2_device_window(wl)
dev = torch.device("cuda:0")
tg = torch.from_numpy(gid).to(dev)
tw = torch.from_numpy(words.reshape(-1).view(np.int64)).to(dev)
tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
v.ingest_device(len(lsn), words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(),
                wl.params["end_lsn"])
torch.cuda.synchronize()
arrs = NativeCurRangeArrs(wl.readsets)
tag = ",".join(k for k in ("HSC_NO_PRE_ASSEMBLE", "HSC_NO_STREAM_PRIO") if k in os.environ) or "default"
for threads in (64, 256):
    for rep in range(4):
        _, st = v.concurrent_check(arrs, nthreads=threads)
        keep = {k: (round(x, 1) if isinstance(x, float) else x) for k, x in st.items()
                if k in ("checks_per_s", "lat_p50_us", "lat_p99_us", "mean_batch", "device_pass_us",
                         "gate_us", "handout_us", "busy_frac")}
        print(json.dumps({"variant": tag, "threads": threads, "rep": rep, **keep}), flush=True)
print(json.dumps({"variant": tag, "small": v.small_stats()}), flush=True)
arrs.close()
v.close()
