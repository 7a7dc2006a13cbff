#!/bin/bash
# One serial kernel profile of the fp32 train step (scripts/step_profile.py --serial under rocprofv3 --kernel-trace), the
# full per-kernel list -> gpurun_out/<tag>_train_serial_full.txt
set -o pipefail
tag=${1:-serial}
extra=$2   # e.g. --amp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_serial1 -o run -- \
  python3 scripts/step_profile.py --marker --serial --steps 10 $extra > gpurun_out/${tag}_serial1.log 2>&1 || exit $?
python3 - "$tag" <<'PY'
import sys
sys.path.insert(0, "scripts")
import prof_summary as P
tag = sys.argv[1]
rows = P.rows_from_trace(f"gpurun_out/{tag}_serial1/run_kernel_trace.csv")
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6 / 10
cat = {}
with open(f"gpurun_out/{tag}_train_serial_full.txt", "w") as f:
    f.write(f"every kernel of scripts/step_profile.py --marker --serial --steps 10 ({tag}): {tot:.2f} ms/step\n")
    f.write("  ms/step  calls/step   avg us  kernel\n")
    for r in rows:
        ms = float(r["TotalDurationNs"]) / 1e6 / 10
        c = int(r["Calls"]) / 10
        n = r["Name"]
        k = n.split("hyres::", 1)[1] if "hyres::" in n else n
        grp = "wgrad" if ("wgrad" in k or "colsum" in k) else "conv" if (k.startswith("conv") or k.startswith("ru_")) else "other"
        cat[grp] = cat.get(grp, 0) + ms
        f.write(f"{ms:9.3f} {c:11.1f} {ms * 1000 / c:8.1f}  {n[:150]}\n")
    f.write("by group (ms/step): " + ", ".join(f"{k} {v:.3f}" for k, v in sorted(cat.items())) + "\n")
print(open(f"gpurun_out/{tag}_train_serial_full.txt").read().splitlines()[-1])
PY
