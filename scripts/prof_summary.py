"""Summarise a rocprofv3 --kernel-trace --stats CSV into a short per-kernel table (ms per step).

    python scripts/prof_summary.py <..._kernel_stats.csv> <steps in the profiled run>
"""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot_ns = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total GPU kernel time {tot_ns / 1e6:.2f} ms over the run ({tot_ns / 1e6 / steps:.2f} ms/step, {steps:g} steps)")
print(f"{'ms/step':>9} {'%':>6} {'calls/step':>10} {'avg us':>9}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    t_ns = float(r["TotalDurationNs"])
    if t_ns / tot_ns < 0.002:
        continue
    print(f"{t_ns / 1e6 / steps:9.3f} {100 * t_ns / tot_ns:6.2f} {int(r['Calls']) / steps:10.1f} "
          f"{float(r['AverageNs']) / 1e3:9.1f}  {r['Name'][:100]}")
