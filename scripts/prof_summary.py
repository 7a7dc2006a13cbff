"""Summarise a rocprofv3 --kernel-trace --stats run into a short per-kernel table (ms per step).

    python scripts/prof_summary.py <..._kernel_stats.csv | ..._results.db | ..._kernel_trace.csv> <steps> [--csv out.csv]

A ``*_kernel_trace.csv`` (rocprofv3 --kernel-trace --output-format csv) of ``scripts/step_profile.py --marker`` is
aggregated over the dispatches AFTER the marker (torch's spin kernel between warm-up and the timed steps) only, so
``calls/step`` counts the replayed steps alone — the stats CSV also holds the capture's eager warm-up passes.

Accepts either the CSV written with ``--output-format csv`` or the rocpd SQLite database that
rocprofv3 writes by default; ``--csv`` re-exports a .db as a kernel_stats CSV (same columns as
rocprofv3's own: Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs).
"""
import csv
import sqlite3
import sys


def rows_from_db(path):
    con = sqlite3.connect(path)
    agg = {}
    for name, dur in con.execute("select name, duration from kernels"):
        a = agg.setdefault(name, [0, 0.0, float("inf"), 0.0])
        a[0] += 1
        a[1] += dur
        a[2] = min(a[2], dur)
        a[3] = max(a[3], dur)
    tot = sum(a[1] for a in agg.values())
    out = []
    for name, (calls, total, mn, mx) in agg.items():
        out.append({"Name": name, "Calls": str(calls), "TotalDurationNs": str(int(total)),
                    "AverageNs": f"{total / calls:.3f}", "Percentage": f"{100 * total / tot:.4f}",
                    "MinNs": str(int(mn)), "MaxNs": str(int(mx))})
    out.sort(key=lambda r: -float(r["TotalDurationNs"]))
    return out


def rows_from_trace(path):
    """Per-kernel rows from a kernel trace, dispatches after the last spin/sleep marker kernel only."""
    tr = list(csv.DictReader(open(path)))
    name_k = "Kernel_Name"
    t0_k, t1_k = "Start_Timestamp", "End_Timestamp"
    tr.sort(key=lambda r: int(r[t0_k]))
    marks = [i for i, r in enumerate(tr) if "spin" in r[name_k].lower() or "sleep" in r[name_k].lower()]
    if marks:
        tr = tr[marks[-1] + 1:]
    agg = {}
    for r in tr:
        dur = int(r[t1_k]) - int(r[t0_k])
        a = agg.setdefault(r[name_k], [0, 0.0, float("inf"), 0.0])
        a[0] += 1
        a[1] += dur
        a[2] = min(a[2], dur)
        a[3] = max(a[3], dur)
    tot = sum(a[1] for a in agg.values()) or 1.0
    return [{"Name": n, "Calls": str(c), "TotalDurationNs": str(int(t)), "AverageNs": f"{t / c:.3f}",
             "Percentage": f"{100 * t / tot:.4f}", "MinNs": str(int(mn)), "MaxNs": str(int(mx))}
            for n, (c, t, mn, mx) in agg.items()]


def main():
    args = sys.argv[1:]
    csv_out = None
    if "--csv" in args:
        i = args.index("--csv")
        csv_out = args[i + 1]
        del args[i:i + 2]
    path = args[0]
    steps = float(args[1]) if len(args) > 1 else 1.0
    if path.endswith(".db"):
        rows = rows_from_db(path)
    elif path.endswith("kernel_trace.csv"):
        rows = rows_from_trace(path)
    else:
        rows = list(csv.DictReader(open(path)))
    if csv_out:
        with open(csv_out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    tot_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total GPU kernel time {tot_ns / 1e6:.2f} ms over the run ({tot_ns / 1e6 / steps:.2f} ms/step, "
          f"{steps:g} steps)")
    print(f"{'ms/step':>9} {'%':>6} {'calls/step':>10} {'avg us':>9}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t_ns = float(r["TotalDurationNs"])
        if t_ns / tot_ns < 0.002:
            continue
        print(f"{t_ns / 1e6 / steps:9.3f} {100 * t_ns / tot_ns:6.2f} {int(r['Calls']) / steps:10.1f} "
              f"{float(r['AverageNs']) / 1e3:9.1f}  {r['Name'][:100]}")


if __name__ == "__main__":
    main()
