"""CPU: bench.py's --gpus N dispatch (the driver's scaling runs).  Without a
launcher, --gpus N > 1 runs the in-process multi-GPU context over devices
0..N-1 and must refuse to run -- never print a one-GPU line -- when fewer
GPUs are visible; under torchrun the world size must match --gpus."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""  # no GPU, whatever the host has
    env["HIP_VISIBLE_DEVICES"] = ""
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("n", [2, 8])
def test_gpus_n_without_devices_exits_nonzero(n):
    r = _run(["--gpus", str(n), "--steps", "1", "--warmup", "0", "--no-cpu", "--no-pmc"])
    assert r.returncode == 2, r.stderr[-2000:]
    assert f"bench.py --gpus {n}: only 0 GPU(s) visible" in r.stderr
    for line in r.stdout.splitlines():  # no result line at all
        with pytest.raises(ValueError):
            json.loads(line)


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"],
             {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr[-2000:]
    assert "bench.py --gpus 2 under WORLD_SIZE 4" in r.stderr


def test_multi_line_reports_devices_used():
    """Static check of the line bench_multi prints: n_gpus is the set of
    devices the members ran on (in process) or the world size (torchrun)."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert '"n_gpus": len(set(devs)) if inproc else N' in src
    assert "args.gpus > 1" in src.split("def main():")[1]


def test_config4_gpus_n_without_devices_exits_nonzero():
    """--config 4 --gpus N runs hsc_multi_graph_scc over in-process members on
    devices 0..N-1, or refuses: never a silent one-GPU line."""
    r = _run(["--config", "4", "--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu",
              "--history-txns", "1000"])
    assert r.returncode == 2, r.stderr[-2000:]
    assert "bench.py --gpus 2: only 0 GPU(s) visible" in r.stderr
    for line in r.stdout.splitlines():
        with pytest.raises(ValueError):
            json.loads(line)


def test_config4_gpus_must_match_world_size():
    r = _run(["--config", "4", "--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"],
             {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr[-2000:]
    assert "bench.py --gpus 2 under WORLD_SIZE 4" in r.stderr


def test_multi_line_carries_cpu_baseline_traffic_and_oracle_parity():
    """Static check of bench_multi: the N > 1 line gets the oracle CPU baseline
    on owner 0's read sets (with parity against the merged GPU verdicts) and
    member 0's PMC traffic; bench_graph keeps its CPU baseline at every N."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    multi = src.split("def bench_multi(args):")[1].split("\ndef ")[0]
    assert 'out["cpu_baseline"] = cpu' in multi
    assert 'cpu = cpu_baseline(log, share0, v0, threads' in multi
    assert '"traffic": traffic.get("bytes_per_batch") if traffic else None' in multi
    assert "traffic = pmc_traffic(args, members=N" in multi
    assert 'out["parity"] = ' in multi
    graph = src.split("def bench_graph(args):")[1].split("\ndef ")[0]
    assert 'out["cpu_baseline"] = graph_cpu_baseline(args)' in graph
    assert "if world == 1 and not args.no_cpu" not in graph
