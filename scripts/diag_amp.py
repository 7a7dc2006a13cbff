"""AMP fixture test (tests/test_parity_gpu.py::test_amp_matches_reference_autocast_fixture) under switches, twice each:
fp16 streaming 1x1 (tuning key 8) on / off, branch streams on / off. Prints the test's own lines and the verdict."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"))
sys.path.insert(0, REPO)
import test_parity_gpu as T  # noqa: E402
from hyres_hip import _lib as L  # noqa: E402
from hyres_hip import ops as O  # noqa: E402

CONFIGS = ((1, True),) if "--once" in sys.argv else ((1, True), (1, True)) if "--quick" in sys.argv else ((1, True), (1, True), (0, True), (1, False), (0, False))
for sh, br in CONFIGS:
    old = ctypes.c_int(0)
    L.call("hyres_conv_tuning", 8, sh, ctypes.byref(old))
    O.BranchStreams.enabled = br
    print(f"=== stream_h {sh} branches {br}", flush=True)
    try:
        T.test_amp_matches_reference_autocast_fixture()
        print("PASS", flush=True)
    except AssertionError as e:
        print("FAIL", str(e)[:300], flush=True)
    finally:
        O.BranchStreams.enabled = True
        L.call("hyres_conv_tuning", 8, old.value, None)
