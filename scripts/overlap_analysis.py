"""Contention evidence from a live kernel trace (rocprofv3 --kernel-trace, no PMC: counter collection serialises
dispatches, so a --pmc run cannot see concurrency). For one kernel: per dispatch, the fraction of its duration
that other kernels were running concurrently, which kernels those were, and the mean duration of its dispatches
bucketed by overlap fraction. A kernel whose long dispatches are the overlapped ones is losing CUs to the
concurrent branch, not running slowly on its own.

    python3 scripts/overlap_analysis.py gpurun_out/r2a_fp32/run_kernel_trace.csv \
        --kernel "conv_fwd_kernel<2, 1, 2, 2, 0, false, false>" [--out profiles/x.json]
"""
import argparse
import collections
import csv
import json


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])))
    rows.sort()
    return rows


def short(name):
    return name.replace("void ", "").replace("hyres::", "").split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = load(a.trace)
    mine = [r for r in rows if short(r[2]) == a.kernel]
    assert mine, "kernel not in trace"
    buckets = collections.defaultdict(list)
    by_grid = collections.defaultdict(lambda: collections.defaultdict(list))
    partners = collections.Counter()
    fracs = []
    for s, e, _, grid in mine:
        dur = e - s
        ov = []
        for s2, e2, n2, _ in rows:
            if s2 >= e:
                break
            if e2 <= s or (s2, e2) == (s, e):
                continue
            ov.append((max(s, s2), min(e, e2)))
            partners[short(n2)] += min(e, e2) - max(s, s2)
        ov.sort()
        covered, cur = 0, None
        for x, y in ov:                       # union of overlapped intervals
            if cur is None or x > cur[1]:
                if cur:
                    covered += cur[1] - cur[0]
                cur = [x, y]
            else:
                cur[1] = max(cur[1], y)
        if cur:
            covered += cur[1] - cur[0]
        f = covered / dur
        fracs.append(f)
        buckets[min(int(f * 4), 3)].append(dur / 1e3)
        by_grid[grid]["alone" if f < 0.25 else "shared" if f >= 0.75 else "partial"].append(dur / 1e3)
    total = sum(e - s for s, e, _, _ in mine) / 1e3
    res = {
        "kernel": a.kernel, "trace": a.trace, "dispatches": len(mine),
        "mean_us": total / len(mine), "min_us": min(e - s for s, e, _, _ in mine) / 1e3,
        "mean_overlap_frac": sum(fracs) / len(fracs),
        "by_overlap_frac": {f"[{k / 4:.2f},{(k + 1) / 4:.2f})": {"n": len(v), "mean_us": sum(v) / len(v)}
                            for k, v in sorted(buckets.items())},
        "by_launch_shape (grid threads: mean us, n)": {
            str(g): {k: [round(sum(v) / len(v), 1), len(v)] for k, v in sorted(d.items())}
            for g, d in sorted(by_grid.items())},
        "top_concurrent_kernels_us": {k: v / 1e3 for k, v in partners.most_common(8)},
    }
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
