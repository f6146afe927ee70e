"""Per-call latency of the drop-in entry on a config-2 window (GPU box):
lone hip_bdb_osql_serial_check calls and 64 collector threads, with the
small-batch phase means (hsc_small_stats).  HSC_SMALL_EMPTY=1 in the
environment gives the launch + done-word floor (wrong verdicts)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from comdb2_amd.hsc import NativeCurRangeArrs, Validator  # noqa: E402
from comdb2_amd.workloads import config2  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
from comdb2_amd.workloads import config2_device_window  # noqa: E402

v = Validator(0)
assert v.register_group("t1", 0, 9) == 0
wl = config2(n_commits=int(os.environ.get("LAT_COMMITS", "1000000")), n_txn=20_000, seed=5,
             build_log=False)
gid, words, lsn = config2_device_window(wl)
dev = torch.device("cuda:0")
tg = torch.from_numpy(gid).to(dev)
tw = torch.from_numpy(words.reshape(-1).view(np.int64)).to(dev)
tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
v.ingest_device(len(lsn), words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(),
                wl.params["end_lsn"])
torch.cuda.synchronize()
arrs = NativeCurRangeArrs(wl.readsets)
out = {}
for name, kw in (("lone", dict(nthreads=1, collect=False)),
                 ("c64", dict(nthreads=64)), ("c64_inflight2", dict(nthreads=64, inflight=2)),
                 ("c32", dict(nthreads=32)), ("c128", dict(nthreads=128))):
    _, st = v.concurrent_check(arrs, **kw)
    out[name] = {k: (round(x, 2) if isinstance(x, float) else x) for k, x in st.items()}
    print(name, json.dumps(out[name]), flush=True)
arrs.close()
v.close()
