"""Cross-kernel interference regression tests (DESIGN §4 "Cross-kernel interference").

A side-stream ``bilinear_fwd_kernel<4,false>`` lost loaded values (one 16-lane quarter of a wave, even dwords of its
first two loads) while a wave of ``conv3x3_wres_bf6_kernel`` or ``ru_fused_f16_kernel`` shared its SIMD. Both kernels now
declare the whole VGPR file (hyres_conv_tuning key 9 = 1, the default), so no other kernel's wave can share those SIMDs.
These tests put each persistent 512-thread kernel on the main stream and the library bilinear on a side stream, as the
MultiScaleRefine / AttentionBlock branch streams do (models/layers/enhancement.py:96-103, models/layers/attention.py:
35-47), and check the bilinear bit for bit against the same resampling alone; the unguarded diagnostic build is run too
and its count printed (the sensitivity of the check). Then whole graphed steps at the bench's size run three times with
the branch streams on: fp32 (bf16x6) and AMP training, autocast eval — every replay bit-identical to the first.
"""
import contextlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1) * scale


def _hog(name, D):
    """A callable launching one persistent kernel on the current stream (2 x 256 x 256 maps)."""
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    if name in ("wres_bf6", "wres_f16"):
        half = name == "wres_f16"
        x = O.to_nhwc(_rand((2, 64, 256, 256), 81).to(D))
        if half:
            x = O.Node(x.v.half(), rg=False)
        w = _rand((64, 64, 3, 3), 82, 1 / 24).to(D)
        b = _rand((64,), 83, 0.1).to(D)
        slope = torch.full((1,), 0.25, device=D)

        def run():
            with torch.autocast("cuda", dtype=torch.float16, enabled=half), \
                    (O.f16_region() if half else contextlib.nullcontext()):
                return O.conv2d(None, x, w, b, pad=1, act=L.ACT_PRELU if not half else L.ACT_RELU, slope=slope).v
        return run
    from models.layers.attention import ResidualUnit
    torch.manual_seed(84)
    mod = ResidualUnit(128).to(D).eval()
    xn = O.Node(O.to_nhwc(_rand((2, 128, 256, 256), 85).to(D)).v.half(), rg=False)

    def run():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16), O.f16_region():
            return mod.hip(None, xn).v
    return run


def _beside(name, guard, reps=6):
    """Wrong bilinear outputs over ``reps`` runs of the hog with three side-stream resamplings each."""
    from hyres_hip import _lib as L
    from hyres_hip import refine_ops as R
    from hyres_hip import ops as O
    D = dev()
    lib = L.load()
    old = lib.hyres_conv_tuning(9, guard, None)
    try:
        other = O.to_nhwc(_rand((2, 64, 256, 256), 74).to(D))
        hog = _hog(name, D)
        side = torch.cuda.Stream(device=D)
        with torch.no_grad():
            ref = R.bilinear(None, other, 128, 128, 2.0, 2.0).v.clone()
            y0 = hog().clone()
            torch.cuda.synchronize()
            wrong, hog_changed = 0, 0
            for _ in range(reps):
                fork = torch.cuda.Event()
                fork.record()
                y = hog()
                side.wait_event(fork)
                with torch.cuda.stream(side):
                    got = [R.bilinear(None, other, 128, 128, 2.0, 2.0).v for _ in range(3)]
                torch.cuda.current_stream().wait_stream(side)
                torch.cuda.synchronize()
                wrong += sum(int((g_ != ref).sum()) for g_ in got)
                hog_changed += int((y != y0).sum())
    finally:
        lib.hyres_conv_tuning(9, 1, None)
    return wrong, hog_changed


@pytest.mark.parametrize("name", ["wres_bf6", "ru_fused_f16", "wres_f16"])
def test_persistent_kernel_beside_side_stream_bilinear(name):
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    if name == "wres_bf6":
        assert L.load().hyres_conv_tuning(7, 1, None) == 0  # bf16x6 (the default) must be on
    if name == "ru_fused_f16":
        assert O.RU_FUSED
    wrong, changed = _beside(name, 1)
    # sensitivity: the diagnostic build without the guard (wres_f16 has no unguarded variant)
    unguarded = _beside(name, 0)[0] if name != "wres_f16" else None
    print(f"{name}: side-stream bilinear wrong {wrong} (guarded), {unguarded} (unguarded diagnostic build); "
          f"hog output changed {changed}")
    assert wrong == 0 and changed == 0


def _net(D, train):
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(D)
    return net.train() if train else net.eval()


def _inputs(D, B=16):
    g = torch.Generator().manual_seed(21)
    x = torch.rand((B, 3, 256, 256), generator=g)
    jd = (x + 0.03 * torch.randn((B, 3, 256, 256), generator=g)).clamp(0, 1)
    return x.to(D), jd.to(D)


@pytest.mark.parametrize("amp", [False, True])
def test_graphed_train_step_bs16_bit_identical_run_to_run(amp):
    """The bench's C2 step (bs 16, 256 x 256, branch streams on; STE quantisation so the step is a pure function of its
    inputs) replayed three times: loss and every parameter gradient identical bit for bit to the first replay."""
    from hyres_hip.graphs import CapturedStep
    from hyres_hip.loss import RateDistortionLoss
    D = dev()
    net = _net(D, True)
    x, jd = _inputs(D)
    crit = RateDistortionLoss(lmbda=0.045, alpha=0)
    params = [p for p in net.parameters() if p.requires_grad]

    def zero():
        for p in params:
            if p.grad is not None:
                p.grad.zero_()
    scale = torch.full((1,), 1024.0, device=D) if amp else None
    # the EntropyBottleneck's training likelihood draws noise even with STE quantisation (compressai EntropyBottleneck
    # in training mode, models/checkerboard.py:96): a fixed injected draw makes every replay the same function
    g = torch.Generator().manual_seed(22)
    net.residual_model.noise.injected = {"z": (torch.rand((16, 8, 8, 128), generator=g) - 0.5).to(D),
                                         "y": (torch.rand((16, 32, 32, 192), generator=g) - 0.5).to(D)}
    cap = CapturedStep(net, x, jd, 0.3, noisequant=False, criterion=crit, zero_grad=zero, amp=amp, loss_scale=scale)
    first = None
    try:
        for r in range(3):
            zero()
            c = cap.replay()[1]
            torch.cuda.synchronize()
            cur = [float(c["loss"])] + [p.grad.detach().clone() for p in params]
            if first is None:
                first = cur
                continue
            assert cur[0] == first[0], (r, cur[0], first[0])
            bad = [i for i, (a, b) in enumerate(zip(cur[1:], first[1:])) if not torch.equal(a, b)]
            assert not bad, f"replay {r}: {len(bad)} gradients differ"
    finally:
        net.residual_model.noise.injected = None
        c = None  # the replay's outputs live in the graph's pool: dropped before close()
        cap.close()


def test_graphed_autocast_eval_bs16_bit_identical_run_to_run():
    """Autocast eval (fp16 activations, fused ResidualUnits, branch streams) at bs 16: three replays, x_hat and both
    likelihoods identical bit for bit."""
    from hyres_hip.graphs import CapturedStep
    D = dev()
    net = _net(D, False)
    x, jd = _inputs(D)
    cap = CapturedStep(net, x, jd, 0.3, amp=True)
    first = None
    try:
        for r in range(3):
            out, _ = cap.replay()
            torch.cuda.synchronize()
            cur = [out["x_hat"].clone(), out["likelihoods"]["y"].clone(), out["likelihoods"]["z"].clone()]
            if first is None:
                first = cur
                continue
            assert all(torch.equal(a, b) for a, b in zip(cur, first)), r
    finally:
        out = None
        cap.close()
