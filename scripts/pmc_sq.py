"""Per-dispatch SQ counters of one kernel from a rocprofv3 --pmc pass (kernel trace only), averaged:

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
        SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv \
        -d <dir> -- python3 scripts/conv_micro.py --H 128 --bf6
    python scripts/pmc_sq.py <dir> --kernel conv3x3_wres_bf6 [--mfma-cycles 32]

Reads (MI355X_MICROARCH.md "rocprofv3 PMC slots"): WAIT_ANY (parked at s_waitcnt / barrier) + WAIT_INST_ANY (issue
stalls) + ACTIVE_INST_ANY ~= WAVE_CYCLES (quad-cycles, summed over waves); VALU_MFMA_BUSY_CYCLES in cycles (32 per
v_mfma_f32_32x32x16_bf16), summed over SIMDs; LDS_BANK_CONFLICT / LDS_IDX_ACTIVE in LDS cycles."""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", required=True)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {a.dir}")
    per = {}
    name = None
    for path in files:
        for r in csv.DictReader(open(path)):
            if a.kernel not in r.get("Kernel_Name", ""):
                continue
            name = r["Kernel_Name"]
            key = (path, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            d = per.setdefault(key, {})
            c = r["Counter_Name"]
            d[c] = d.get(c, 0.0) + float(r["Counter_Value"])
    if not per:
        raise SystemExit("kernel not found")
    keys = sorted({c for d in per.values() for c in d})
    avg = {c: sum(d.get(c, 0.0) for d in per.values()) / len(per) for c in keys}
    print(f"{name[:90]}: {len(per)} dispatches, per-dispatch averages")
    for c in keys:
        print(f"  {c:28s} {avg[c]:.4g}")
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in avg:
                print(f"  {c} / WAVE_CYCLES = {avg[c] / wc:.3f}")
    if "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
        print(f"  LDS bank-conflict share = {avg.get('SQ_LDS_BANK_CONFLICT', 0.0) / avg['SQ_LDS_IDX_ACTIVE']:.3f}")


if __name__ == "__main__":
    main()
