"""Replicant coalesce throughput: GPU hsc_coalesce_readsets
(host arrays in and out: upload, kernel, download, compaction) vs the CPU
restatement oracle/coalesce_oracle.c (one core), on config-2-like batches of
many small read sets and on a few very large read sets (with and without the
comparator's tie-with-everything ranges).  Checks equality."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle
from coalesce_model import as_rows, long_run_readsets, random_readsets
from comdb2_amd.hsc import Validator

v = Validator(0)
res = {}
for name, kw in (("100k sets x <=20 ranges", dict(ntxn=100_000, max_ranges=20)),
                 ("8 sets x <=200k ranges, NULL lower keys (tie with everything)",
                  dict(ntxn=8, max_ranges=200_000)),
                 ("8 sets x <=200k ranges, present empty lower keys, no NULL (level-parallel sort)",
                  dict(ntxn=8, max_ranges=200_000, null_lo=0.0)),
                 ("8 sets x 200k ranges, each one long (table, index) run", "long")):
    if len(sys.argv) > 1 and sys.argv[1] not in name:  # case filter (profiling)
        continue
    rs = long_run_readsets(7) if kw == "long" else random_readsets(7, **kw)
    t0 = time.perf_counter(); want = oracle.coalesce(rs); cpu = time.perf_counter() - t0
    v.coalesce(rs)  # warm
    t0 = time.perf_counter(); got = v.coalesce(rs); gpu = time.perf_counter() - t0
    ok = list(got.txn_off) == list(want.txn_off) and np.array_equal(got.rkey_off, want.rkey_off) \
        and np.array_equal(got.islocked, want.islocked) and np.array_equal(got.lkey_off, want.lkey_off)
    n = len(rs.table)
    res[name] = dict(ranges=n, out_ranges=int(got.txn_off[-1]), cpu_s=cpu, gpu_s=gpu,
                     cpu_ranges_per_s=n / cpu, gpu_ranges_per_s=n / gpu, equal=ok)
print(json.dumps(res, indent=1))
