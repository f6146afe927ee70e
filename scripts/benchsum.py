"""One-line summaries of bench.py JSON logs: python scripts/benchsum.py gpurun_out/x.log ..."""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError) as e:
        print(path, "unreadable:", e)
        continue
    c = d.get("config", {})
    print(f"{path}: {d['value'] / 1e6:.1f} M {d['unit']}  {d['ms_per_step'] * 1e3:.1f} us/step"
          f"  serial {c.get('serial_ms_per_step', 0) * 1e3:.1f} us"
          f"  frac {d.get('roofline', {}).get('frac', 0):.3f}  layout {c.get('window_layout')}"
          f"  keys {c.get('window_keys_per_gpu')}  conflicts {c.get('conflict_rate')}"
          f"  ingest {d.get('ingest_ms', 0):.1f} ms  parity {d.get('parity')}"
          f"  imbalance {d.get('imbalance', {}).get('time_max_over_mean')}")
