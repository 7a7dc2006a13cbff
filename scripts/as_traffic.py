"""HBM bytes of the north-star analysis + synthesis pass (g_a on the residual, g_s on y_hat; BASELINE.json
north_star, models/checkerboard.py:35-58) at bs 16 x 256^2, from rocprofv3 PMC counters instead of the
SURVEY §8d ledger.

Workload (run it under two separate PMC passes):
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir_f> -o run -- python3 scripts/as_traffic.py
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d <dir_w> -o run -- python3 scripts/as_traffic.py
Summary:
    python3 scripts/as_traffic.py --summarize <dir_f> <dir_w> [--ms <graph-replay ms per pass>] --out file.json

The workload runs one warm-up pass (weight re-layouts happen there), a torch spin kernel as a delimiter, then PASSES eager
passes of g_a + g_s; only the dispatches after the marker count.  Bytes per pass = (2 x FETCH_SIZE +
WRITE_SIZE) KiB x 1024 / PASSES (gfx950: FETCH_SIZE reads half of a wide coalesced read,
MI355X_MICROARCH.md "HBM"; Infinity-Cache hits are counted, so this is an upper bound on DRAM bytes).
"""
import argparse
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = 4


def workload():
    sys.path[:0] = [os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"), REPO]
    import torch
    from hyres_hip import ops as O
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    dev = torch.device("cuda:0")
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).eval()
    rm = net.residual_model
    B, H, W = 16, 256, 256
    g = torch.Generator().manual_seed(1926)
    x = (torch.randint(0, 256, (B, 3, H, W), generator=g).float() / 255.0).to(dev)
    with torch.no_grad():
        xn = O.to_nhwc(x - 0.5, rg=False)
        yh = O.Node.new(B, H // 8, W // 8, rm.M, dev, rg=False)
        yh.v.copy_(torch.randn(yh.v.shape, generator=torch.Generator().manual_seed(3)).to(dev))
        rm.g_a.hip(None, xn)
        rm.g_s.hip(None, yh)
        torch.cuda.synchronize()
        torch.cuda._sleep(1000)  # delimiter dispatch (a "spin" kernel)
        torch.cuda.synchronize()
        for _ in range(PASSES):
            rm.g_a.hip(None, xn)
            rm.g_s.hip(None, yh)
        torch.cuda.synchronize()


def _rows(d, counter):
    out = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") == counter:
                out.append((int(r.get("Dispatch_Id") or r.get("Correlation_Id")), r["Kernel_Name"], float(r["Counter_Value"])))
    per = {}
    for did, name, v in out:
        k = per.setdefault(did, [name, 0.0])
        k[1] += v
    return per


def summarize(dir_f, dir_w, ms, out):
    tot = {}
    for counter, d in (("FETCH_SIZE", dir_f), ("WRITE_SIZE", dir_w)):
        per = _rows(d, counter)
        marks = [did for did, (name, _) in per.items() if "spin" in name.lower() or "sleep" in name.lower()]
        start = max(marks) if marks else -1  # the delimiter before the measured passes
        hy = {did: v for did, v in per.items() if did > start}
        tot[counter] = sum(v for _, v in hy.values())
        tot[counter + "_dispatches"] = len(hy)
    fetch = 2.0 * tot["FETCH_SIZE"] * 1024 / PASSES
    write = tot["WRITE_SIZE"] * 1024 / PASSES
    res = {"what": "analysis + synthesis pass (g_a + g_s forward), bs 16, 256x256, fp32",
           "bytes_per_pass": fetch + write, "fetch_bytes_per_pass": fetch, "write_bytes_per_pass": write,
           "dispatches_per_pass": tot["FETCH_SIZE_dispatches"] / PASSES,
           "ledger_bytes_per_pass": 16 * 1.836e9,
           "method": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes), 2 x FETCH_SIZE + WRITE_SIZE, KiB"}
    if ms:
        res["ms_per_pass_graph"] = ms
        res["hbm_gbs"] = round(res["bytes_per_pass"] / (ms * 1e-3) / 1e9, 1)
        res["hbm_frac"] = round(res["bytes_per_pass"] / (ms * 1e-3) / 8e12, 4)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--summarize":
        ap = argparse.ArgumentParser()
        ap.add_argument("--summarize", nargs=2)
        ap.add_argument("--ms", type=float, default=None)
        ap.add_argument("--out", required=True)
        a = ap.parse_args()
        summarize(a.summarize[0], a.summarize[1], a.ms, a.out)
    else:
        workload()
