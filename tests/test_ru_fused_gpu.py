"""The fused ResidualUnit / ResidualBottleneckBlock inference kernel (csrc/ru_fused.hip, ``hyres_ru_fused_f16``).

Reference semantics: models/layers/attention.py:11-30 (ResidualUnit: relu(x + conv1x1(relu(conv3x3(relu(conv1x1(x))))))),
compressai's ResidualBottleneckBlock (the same without the final ReLU), under torch.autocast(float16) with fp16
activations (BASELINE configs[4]). The fused kernel keeps t1 / t2 on chip but rounds them to fp16 exactly where the
unfused path stores them, and every GEMM takes fp16 operands as before, so:
  * against torch (float64) with those rounding points: within one fp16 ulp of the output (2e-3 max-norm);
  * against this build's unfused three-conv path: the same bound (only fp32 summation order differs);
  * the whole autocast eval forward with the fused kernel on vs off: PSNR within 0.01 dB, bits within 0.5 %.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from helpers import rel_err

pytestmark = pytest.mark.gpu


def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1) * scale


def _torch_ru(x, ws, bs, final_relu):
    """float64 reference with the HIP path's fp16 rounding points (operands of every GEMM, t1, t2, y)."""
    def r16(t):
        return t.half().double()
    xd = r16(x.double())
    t1 = r16(F.relu(F.conv2d(xd, r16(ws[0].double()), bs[0].double())))
    t2 = r16(F.relu(F.conv2d(t1, r16(ws[1].double()), bs[1].double(), padding=1)))
    y = F.conv2d(t2, r16(ws[2].double()), bs[2].double()) + xd
    if final_relu:
        y = F.relu(y)
    return r16(y).float()


@pytest.mark.parametrize("final_relu", [True, False])
@pytest.mark.parametrize("B,H,W", [(2, 32, 64), (2, 30, 128), (1, 8, 192)])
def test_ru_fused_matches_torch_and_unfused(B, H, W, final_relu, monkeypatch):
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    from hyres_hip.layers import ResidualBottleneckBlock
    from models.layers.attention import ResidualUnit
    D = dev()
    N = 128
    torch.manual_seed(7)
    mod = (ResidualUnit(N) if final_relu else ResidualBottleneckBlock(N, N)).to(D).eval()
    convs = ([mod.conv[0], mod.conv[2], mod.conv[4]] if final_relu else [mod.conv1, mod.conv2, mod.conv3])
    with torch.no_grad():  # non-trivial biases
        for i, c in enumerate(convs):
            c.bias.copy_(_rand(c.bias.shape, 40 + i, 0.1).to(D))
    x = _rand((B, N, H, W), 11).to(D)
    ref = _torch_ru(x.cpu(), [c.weight.detach().cpu() for c in convs], [c.bias.detach().cpu() for c in convs],
                    final_relu)
    assert L.load().hyres_ru_fused_f16_ok(B, H, W, N)
    outs = {}
    for fused in (True, False):
        monkeypatch.setattr(O, "RU_FUSED", fused)
        xn = O.to_nhwc(x)
        xn = O.Node(xn.v.half(), rg=False)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16), O.f16_region():
            yn = mod.hip(None, xn)
        assert yn.half
        outs[fused] = O.to_nchw(yn).cpu()
    torch.cuda.synchronize()
    e_ref, e_unf = rel_err(outs[True], ref), rel_err(outs[True], outs[False])
    print(f"B{B} H{H} W{W} relu={final_relu}: fused vs torch {e_ref:.2e}, vs unfused {e_unf:.2e}, "
          f"unfused vs torch {rel_err(outs[False], ref):.2e}")
    assert e_ref < 2e-3 and e_unf < 2e-3


def test_ru_fused_eval_forward_matches_unfused(monkeypatch):
    """ResidualJPEGCompression eval forward under autocast (fp16 activations): every ResidualUnit of the
    AttentionBlock(N)s and every RBB runs fused (128-channel maps, W % 64 == 0) — the same x_hat / likelihoods as the
    unfused path up to fp16 summation-order effects."""
    from hyres_hip import ops as O
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    D = dev()
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(D).eval()
    g = torch.Generator().manual_seed(5)
    x = torch.rand((2, 3, 256, 256), generator=g)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(O, "RU_FUSED", fused)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            out = net(x)
        torch.cuda.synchronize()
        mse = float(F.mse_loss(out["x_hat"].double().cpu(), x.double()))
        bits = float(sum((-torch.log2(v.double())).sum() for v in out["likelihoods"].values()))
        res[fused] = (10 * math.log10(1.0 / mse), bits)
    dpsnr = res[True][0] - res[False][0]
    dbits = res[True][1] / res[False][1] - 1
    print(f"fused vs unfused eval: dPSNR {dpsnr:.5f} dB, bits {dbits:.2e}")
    assert abs(dpsnr) < 0.01 and abs(dbits) < 5e-3


@pytest.mark.parametrize("final_relu", [True, False])
def test_ru_fused_amp_training_matches_unfused(final_relu, monkeypatch):
    """AMP training (fp16 activations and gradients inside an f16_region): the fused forward also writes t1 / t2 and
    records the three convs' backward; output, input gradient and every weight / bias gradient match the unfused
    chain up to fp32 summation order (a ReLU decision at an fp16 tie may flip: normwise 1e-2)."""
    from hyres_hip import ops as O
    from hyres_hip.layers import ResidualBottleneckBlock
    from models.layers.attention import ResidualUnit
    D = dev()
    N, B, H, W = 128, 2, 16, 64
    torch.manual_seed(9)
    mod = (ResidualUnit(N) if final_relu else ResidualBottleneckBlock(N, N)).to(D).train()
    x = _rand((B, N, H, W), 12).to(D)
    gy = _rand((B, N, H, W), 13).half().float().to(D)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(O, "RU_FUSED", fused)
        for p in mod.parameters():
            p.grad = None
        tape = O.Tape()
        xn = O.to_nhwc(x, rg=True)
        xn = O.Node(xn.v.half(), rg=True)
        with torch.autocast("cuda", dtype=torch.float16), O.f16_region():
            yn = mod.hip(tape, xn)
        assert yn.half
        y = O.to_nchw(yn)
        yn.set_grad(O.nchw_grad_to_nhwc(gy))
        tape.backward()
        torch.cuda.synchronize()
        res[fused] = [y.cpu(), O.to_nchw_grad(xn).cpu()] + [p.grad.detach().cpu().clone() for p in mod.parameters()]
    errs = [rel_err(a, b) for a, b in zip(res[True], res[False])]
    print("fused vs unfused (y, gx, params):", ["%.1e" % e for e in errs])
    assert errs[0] < 2e-3
    assert max(errs[1:]) < 1e-2
