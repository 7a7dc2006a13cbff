"""Concurrency of a replayed step from a rocprofv3 kernel trace (the dispatches after the last spin/sleep marker,
scripts/step_profile.py --marker): wall time, time with >= 1 kernel running (busy), idle gaps, and per kernel its
total time and its SOLO time (no other kernel running) — the solo time is what a kernel adds to the step's critical
path directly; overlapped time is shared with the concurrent branches.

    python scripts/trace_overlap.py gpurun_out/r4d_fp32/run_kernel_trace.csv [steps=10] [top=25]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    tr = list(csv.DictReader(open(path)))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(tr) if "spin" in r["Kernel_Name"].lower() or "sleep" in r["Kernel_Name"].lower()]
    if marks:
        tr = tr[marks[-1] + 1:]
    ev = []
    for i, r in enumerate(tr):
        ev.append((int(r["Start_Timestamp"]), 1, i))
        ev.append((int(r["End_Timestamp"]), -1, i))
    ev.sort(key=lambda e: (e[0], e[1]))
    running = set()
    last = ev[0][0]
    busy = 0
    solo = {}
    conc_hist = {}
    for t, d, i in ev:
        dt = t - last
        if dt > 0:
            n = len(running)
            conc_hist[n] = conc_hist.get(n, 0) + dt
            if n:
                busy += dt
            if n == 1:
                k = tr[next(iter(running))]["Kernel_Name"]
                solo[k] = solo.get(k, 0) + dt
        last = t
        if d > 0:
            running.add(i)
        else:
            running.discard(i)
    wall = ev[-1][0] - ev[0][0]
    tot = {}
    cnt = {}
    for r in tr:
        k = r["Kernel_Name"]
        tot[k] = tot.get(k, 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        cnt[k] = cnt.get(k, 0) + 1
    print(f"{len(tr)} dispatches over {steps:g} steps: wall {wall / steps / 1e6:.3f} ms/step, busy (>= 1 kernel) "
          f"{busy / steps / 1e6:.3f}, idle {(wall - busy) / steps / 1e6:.3f}, kernel time {sum(tot.values()) / steps / 1e6:.3f}")
    print("  time by number of concurrent kernels (ms/step): " +
          ", ".join(f"{n}: {v / steps / 1e6:.2f}" for n, v in sorted(conc_hist.items())))
    print(f"  {'solo ms/step':>12} {'total ms/step':>13} {'calls/step':>10}  kernel")
    for k in sorted(tot, key=lambda k: -solo.get(k, 0))[:top]:
        print(f"  {solo.get(k, 0) / steps / 1e6:12.3f} {tot[k] / steps / 1e6:13.3f} {cnt[k] / steps:10.1f}  {k[:100]}")


if __name__ == "__main__":
    main()
