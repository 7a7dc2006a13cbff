"""Probe (round 5): dilation-2 3x3 conv input gradient at 1x256x384 with the epilogue pieces toggled one at a time."""
import sys, torch
sys.path.insert(0, "/root/repo/hyres-residual-enhanced-hybrid-image-compression_amd"); sys.path.insert(0, "/root/repo/tests")
import torch.nn.functional as F
from hyres_hip import _lib as L, ops as O
from helpers import rel_err
D = torch.device("cuda:0")
B, H, W, C, dil = 1, 256, 384, 64, 2
g = torch.Generator().manual_seed(1)
x = torch.randn(B, C, H, W, generator=g); w = torch.randn(C, C, 3, 3, generator=g) / 24; gy = torch.randn(B, C, H, W, generator=g)
b = torch.randn(C, generator=g) * 0.1; r = torch.randn(B, C, H, W, generator=g)
for (use_b, use_r, r_rg, act) in [(0, 0, 0, 0), (1, 0, 0, 0), (0, 1, 0, 0), (0, 1, 1, 0), (0, 0, 0, 1), (1, 1, 0, 1), (1, 1, 1, 1)]:
    xr = x.double().requires_grad_()
    pre = F.conv2d(xr, w.double(), b.double() if use_b else None, padding=dil, dilation=dil)
    if use_r:
        pre = pre + r.double()
    yr = F.relu(pre) if act else pre
    yr.backward(gy.double())
    tape = O.Tape(); xn = O.to_nhwc(x.to(D), rg=True)
    rn = O.to_nhwc(r.to(D), rg=bool(r_rg)) if use_r else None
    yn = O.conv2d(tape, xn, torch.nn.Parameter(w.to(D)), b.to(D) if use_b else None, pad=dil, dil=dil,
                  act=L.ACT_RELU if act else L.ACT_NONE, res=rn)
    yn.set_grad(O.nchw_grad_to_nhwc(gy.to(D))); tape.backward(); torch.cuda.synchronize()
    print("bias", use_b, "res", use_r, "res.rg", r_rg, "relu", act, "y", "%.2e" % rel_err(O.to_nchw(yn).double().cpu(), yr.detach()),
          "dx", "%.2e" % rel_err(O.to_nchw_grad(xn).double().cpu(), xr.grad), flush=True)
