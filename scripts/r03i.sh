#!/bin/bash
# Append-path check: the incremental-window GPU tests (appends, folds, new
# groups, raw logs, streams), then config 1 (the commit stream).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03i}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_new_groups.py tests/test_gpu_recon.py tests/test_gpu_streams.py tests/test_gpu_small.py tests/test_gpu_ctiles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 400 python3 bench.py --config 1 > gpurun_out/${T}_config1.log 2> gpurun_out/${T}_config1.err || { tail -20 gpurun_out/${T}_config1.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_config1.log').read().strip().splitlines()[-1])
print(d['value'], d['check_us'], d['append_us_per_commit'], d['parity_with_oracle_golden'], d['cpu_baseline']['value'], json.dumps(d['fold_every_1k_commits']))"
echo r03i done
