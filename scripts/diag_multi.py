"""Diagnostic: a multi context vs one context on a random log taken in pieces
(tests/test_gpu_multi.py::test_random_logs_appended_in_pieces), after every
append, with auto splitters and with everything on member 0."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import torch  # noqa: E402,F401  (HIP initialised by torch first, as the tests do)

from comdb2_amd.hsc import MultiValidator, Validator  # noqa: E402
from comdb2_amd.workloads import random_case  # noqa: E402
from test_incremental import log_slice  # noqa: E402


def run(n, seed, everything_on_0):
    log, rs = random_case(800 + seed, n_commits=150, n_txn=50)
    rng = np.random.default_rng(seed)
    cuts = sorted(set(rng.integers(1, log.nrec, size=5).tolist()))
    pieces = [0] + cuts + [log.nrec]
    m = MultiValidator([0] * n)
    one = Validator(0)
    if everything_on_0:
        m.set_splitters(np.full(n - 1, 0xFFFFFFFF, np.uint32), np.full((8, n - 1), ~np.uint64(0)))
    m.ingest_log(log_slice(log, 0, pieces[1]))
    one.ingest_log(log_slice(log, 0, pieces[1]))
    a0, b0 = m.check_readsets(rs) != 0, one.check_readsets(rs) != 0
    print(f"n {n} seed {seed} on0 {everything_on_0} piece 0: diff {np.nonzero(a0 != b0)[0].tolist()}")
    for k, (a, b) in enumerate(zip(pieces[1:], pieces[2:])):
        m.append_log(log_slice(log, a, b))
        one.append_log(log_slice(log, a, b))
        x, y = m.check_readsets(rs) != 0, one.check_readsets(rs) != 0
        d = np.nonzero(x != y)[0].tolist()
        print(f"  piece {k + 1} [{a},{b}): diff {d} multi {x[d].tolist()} one {y[d].tolist()} "
              f"stats {m.multi_stats()} delta {[m.member(i).delta_rows for i in range(n)]}")
    m.close()
    one.close()


for seed in range(4):
    for n in (2, 4):
        for on0 in (False, True):
            run(n, seed, on0)
