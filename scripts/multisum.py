"""Summarise bench_multi JSON lines (the multi-GPU legs) from log files."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "device_routed" not in d:
            continue
        dr, r = d["device_routed"], d["routing"]
        print(f"{f}: value {d['value']:.4g} ms {d['ms_per_step']:.4f} serial "
              f"{d['config']['serial_ms_per_step']:.4f} frac {d['roofline']['frac']:.3f} | device-routed ms "
              f"{dr['ms_per_step']:.4f} serial {dr['serial_ms_per_step']:.4f} | enqueue us "
              f"{r.get('host_enqueue_us_per_step')} | imbalance {d['imbalance']['max_over_mean']:.3f} "
              f"member ms {[round(x, 4) for x in d['imbalance']['member_probe_ms']]} | equal "
              f"{r['verdicts_equal_device_routed']}")
        if "api" in d:
            a = d["api"]
            for k, st in a["concurrent_callers"].items():
                print(f"   api {k}: {st.get('checks_per_s', 0):.4g}/s p50 {st['lat_p50_us']:.1f} "
                      f"p99 {st['lat_p99_us']:.1f} busy {st.get('busy_frac')} parity "
                      f"{st['parity_with_device_batch']}")
            print("   members/call", a["members_per_call"], "route us", a["host_route_us_per_call"],
                  "launch us", a.get("host_launch_us_per_call"), "wait us", a.get("wait_us_per_call"),
                  "front lock us", a.get("front_small_stats", {}).get("lock_us"))
