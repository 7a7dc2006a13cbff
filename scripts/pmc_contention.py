"""Counter-level view of the dominant conv kernel in the live step (concurrent branch streams) vs the same
step with the branches serialised (HYRES_BRANCH_MAX_PIXELS=0): per-dispatch averages of the SQ / GRBM
counters of one rocprofv3 --pmc pass each (scripts/pmc_contention.sh).

    python scripts/pmc_contention.py <live_dir> <serial_dir> --kernel 'conv_fwd_kernel<2, 1, 2, 2, 0, false, false>'
"""
import argparse
import csv
import glob
import json
import os


def load(d, kernel):
    rows = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel not in r.get("Kernel_Name", ""):
                continue
            key = (path, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            e = rows.setdefault(key, {})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    n = len(rows)
    if not n:
        return {"dispatches": 0}
    avg = {}
    for e in rows.values():
        for k, v in e.items():
            avg[k] = avg.get(k, 0.0) + v / n
    avg["dispatches"] = n
    return avg


def derived(a):
    out = dict(a)
    wc = a.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        # SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES (MI355X_MICROARCH.md, PMC slots)
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in a:
                out[k + "_frac_of_wave_cycles"] = round(a[k] / wc, 4)
    if a.get("SQ_BUSY_CYCLES") and a.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        out["mfma_busy_per_busy_cycle"] = round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / a["SQ_BUSY_CYCLES"], 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("live")
    ap.add_argument("serial")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {"kernel": a.kernel, "live": derived(load(a.live, a.kernel)), "serial": derived(load(a.serial, a.kernel))}
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
