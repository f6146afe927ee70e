"""Golden verdicts of BASELINE config 1: the full 10k-txn commit stream of
comdb2_amd.workloads.config1_events (tests/tools/serial.c shaped, seed
0xC0FFEE01) replayed through the oracle (oracle/serial_oracle.c, the CPU
restatement of bdb_osql_serial_check), one check per commit against the whole
log so far, each passing write txn logged before the next commit
(SURVEY.md §7 hard part 7a).  Writes tests/golden/config1_replay.json:
{"seed", "n_txn", "rc": {txn name: rc}} -- the oracle replay is quadratic in
the log (minutes), the GPU test replays incrementally and compares.

    python tests/golden/make_config1_replay.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from comdb2_amd.workloads import SEED_CONFIG1, config1_events, replay  # noqa: E402


def main(n_txn: int = 10_000, out: str = os.path.join(HERE, "config1_replay.json")):
    ev = config1_events(seed=SEED_CONFIG1, n_txn=n_txn)
    rc = replay(ev, lambda log, rs: oracle.check(log, rs)[0])
    json.dump({"seed": SEED_CONFIG1, "n_txn": n_txn, "checked": len(rc),
               "not_serializable": int(sum(v != 0 for v in rc.values())),
               "rc": {k: int(v) for k, v in rc.items()}}, open(out, "w"))
    print(f"{len(rc)} checks, {sum(v != 0 for v in rc.values())} not serializable -> {out}")


if __name__ == "__main__":
    main()
