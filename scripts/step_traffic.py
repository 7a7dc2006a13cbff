"""HBM bytes of one whole C2 train step (every kernel of the graph replay + optimiser tail) from two rocprofv3 PMC
passes over scripts/step_profile.py --marker, against the step time: the step-level HBM utilisation beside the
per-kernel rooflines of the bench line.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir_f> -o run -- python3 scripts/step_profile.py --marker [--amp]
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d <dir_w> -o run -- python3 scripts/step_profile.py --marker [--amp]
    python3 scripts/step_traffic.py <dir_f> <dir_w> --steps 10 --ms <ms/step> --what "..." --out file.json

Bytes per step = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 / steps over the dispatches after the marker (gfx950:
FETCH_SIZE counts half of a wide coalesced read, MI355X_MICROARCH.md "HBM"; narrow reads are then over-counted, and
Infinity-Cache hits are included, so the corrected figure is an upper bound; the raw 1 x FETCH_SIZE one a lower bound).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from as_traffic import _rows  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--ms", type=float, required=True, help="ms per step of an unprofiled run")
    ap.add_argument("--what", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    tot = {}
    for counter, d in (("FETCH_SIZE", a.fetch_dir), ("WRITE_SIZE", a.write_dir)):
        per = _rows(d, counter)
        marks = [did for did, (name, _) in per.items() if "spin" in name.lower() or "sleep" in name.lower()]
        start = max(marks) if marks else -1
        after = {did: v for did, v in per.items() if did > start}
        tot[counter] = sum(v for _, v in after.values()) * 1024 / a.steps
        tot[counter + "_dispatches"] = len(after) / a.steps
    hi = 2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]
    lo = tot["FETCH_SIZE"] + tot["WRITE_SIZE"]
    sec = a.ms * 1e-3
    res = {"what": a.what, "ms_per_step": a.ms, "dispatches_per_step": tot["FETCH_SIZE_dispatches"],
           "fetch_size_bytes_per_step_raw": tot["FETCH_SIZE"], "write_bytes_per_step": tot["WRITE_SIZE"],
           "hbm_bytes_per_step_upper": hi, "hbm_bytes_per_step_lower": lo,
           "hbm_tbs_upper": round(hi / sec / 1e12, 3), "hbm_tbs_lower": round(lo / sec / 1e12, 3),
           "hbm_frac_upper": round(hi / sec / 8e12, 4), "hbm_frac_lower": round(lo / sec / 8e12, 4),
           "method": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) over scripts/step_profile.py --marker"}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
