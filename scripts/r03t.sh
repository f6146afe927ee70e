#!/bin/bash
# Round-3 check of the one-pass narrow descent (key and max trees read
# together) and the small stage marshalled in place: the narrow / small /
# collector / parity GPU tests, the latency legs (lone call, collector) and
# the config-2 bench API leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03t}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_small.py tests/test_collector.py \
  tests/test_gpu_streams.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 300 python3 scripts/latency.py > gpurun_out/${T}_latency.log 2> gpurun_out/${T}_latency.err || { tail gpurun_out/${T}_latency.err; exit 1; }
cat gpurun_out/${T}_latency.log
timeout -k 10 400 python3 bench.py --no-cpu --no-pmc > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
python3 scripts/benchsum.py gpurun_out/${T}_bench.log
python3 - gpurun_out/${T}_bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(json.dumps(d.get("api"), indent=None)[:1500])
PY
echo r03t done
