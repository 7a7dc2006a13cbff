"""Summarise a rocprofv3 --kernel-trace --stats run into a short per-kernel table (ms per step).

    python scripts/prof_summary.py <..._kernel_stats.csv | ..._results.db> <steps> [--csv out.csv]

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


def main():
    args = sys.argv[1:]
    csv_out = None
    if "--csv" in args:
        i = args.index("--csv")
        csv_out = args[i + 1]
        del args[i:i + 2]
    path = args[0]
    steps = float(args[1]) if len(args) > 1 else 1.0
    rows = rows_from_db(path) if path.endswith(".db") else list(csv.DictReader(open(path)))
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
