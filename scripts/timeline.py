"""Concurrency of a replayed step from a rocprofv3 kernel trace (scripts/step_profile.py --marker run): per queue busy
time, the union of all kernels' intervals (time the GPU runs anything), and the wall span, per step.

    python scripts/timeline.py <run_kernel_trace.csv> <steps>
"""
import csv
import sys
from collections import defaultdict


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    tr = list(csv.DictReader(open(path)))
    last = max((i for i, r in enumerate(tr) if "spin" in r["Kernel_Name"].lower() or "sleep" in r["Kernel_Name"].lower()),
               default=-1)
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"]) for r in tr[last + 1:]]
    ks.sort()
    t0, t1 = ks[0][0], max(e for _, e, _, _ in ks)
    wall = (t1 - t0) / 1e6 / steps
    busy = defaultdict(int)
    for s, e, q, _ in ks:
        busy[q] += e - s
    # union of intervals
    uni, cs, ce = 0, None, None
    for s, e, _, _ in ks:
        if cs is None or s > ce:
            if cs is not None:
                uni += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    uni += ce - cs
    # time with >= 2 kernels running
    ev = sorted([(s, 1) for s, _, _, _ in ks] + [(e, -1) for _, e, _, _ in ks])
    depth, prev, multi = 0, ev[0][0], 0
    for t, d in ev:
        if depth >= 2:
            multi += t - prev
        depth += d
        prev = t
    print(f"{len(ks) / steps:.0f} kernels/step, wall span {wall:.2f} ms/step, GPU busy (union) {uni / 1e6 / steps:.2f} ms/step "
          f"({uni / (t1 - t0):.3f}), >= 2 kernels running {multi / 1e6 / steps:.2f} ms/step, "
          f"sum of durations {sum(busy.values()) / 1e6 / steps:.2f} ms/step")
    for q, b in sorted(busy.items(), key=lambda kv: -kv[1]):
        n = sum(1 for _, _, qq, _ in ks if qq == q)
        print(f"  queue {q}: {b / 1e6 / steps:.2f} ms/step busy, {n / steps:.0f} kernels/step")


if __name__ == "__main__":
    main()
