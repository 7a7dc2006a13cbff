"""Debug: the 1x1 epilogue chain of tests/test_parity_gpu.py at one size; reports every tensor's error."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"), os.path.join(REPO, "tests")]
import torch
import torch.nn.functional as F
from helpers import rel_err


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1) * scale


def main(B, H, W, C0, C1, C2):
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    x = _rand((B, C0, H, W), 11)
    r = _rand((B, C1, H, W), 12)
    ws = [_rand(sh, 13 + i, 1.0 / sh[1] ** 0.5) for i, sh in
          enumerate([(C1, C0, 1, 1), (C0, C1, 1, 1), (C2, C0, 1, 1), (C2, C0, 1, 1)])]
    bs = [_rand((sh,), 20 + i, 0.1) for i, sh in enumerate([C1, C0, C2, C2])]
    xr, rr = x.clone().requires_grad_(), r.clone().requires_grad_()
    wr = [w.clone().requires_grad_() for w in ws]
    br = [b.clone().requires_grad_() for b in bs]
    a = F.relu(F.conv2d(xr, wr[0], br[0]) + rr)
    b_ = F.relu(F.conv2d(a, wr[1], br[1]))
    c_ = F.conv2d(b_, wr[2], br[2])
    yr = c_ + F.conv2d(xr, wr[3], br[3])
    for t in (a, b_, c_):
        t.retain_grad()
    gy = _rand(yr.shape, 30)
    yr.backward(gy)
    D = torch.device("cuda:0")
    wd = [torch.nn.Parameter(w.to(D)) for w in ws]
    bd = [torch.nn.Parameter(b.to(D)) for b in bs]
    tape = O.Tape()
    xn = O.to_nhwc(x.to(D), rg=True)
    rn = O.to_nhwc(r.to(D), rg=True)
    an = O.conv2d(tape, xn, wd[0], bd[0], act=L.ACT_RELU, res=rn)
    bn = O.conv2d(tape, an, wd[1], bd[1], act=L.ACT_RELU)
    cn = O.conv2d(tape, bn, wd[2], bd[2])
    yn = O.conv2d(tape, xn, wd[3], bd[3], res=cn)
    print("fwd a", rel_err(O.to_nchw(an).cpu(), a), "b", rel_err(O.to_nchw(bn).cpu(), b_), "y",
          rel_err(O.to_nchw(yn).cpu(), yr))
    yn.set_grad(O.nchw_grad_to_nhwc(gy.to(D)))
    tape.backward()
    torch.cuda.synchronize()
    ga = (a.grad * (a > 0)).detach()
    print("an._g (masked) vs torch pre-act grad", rel_err(an._g.permute(0, 3, 1, 2).cpu(), ga), "gmasked", an.gmasked,
          "bn._g", rel_err(bn._g.permute(0, 3, 1, 2).cpu(), (b_.grad * (b_ > 0)).detach()) if bn._g is not None else None)
    print("grad x", rel_err(O.to_nchw_grad(xn).cpu(), xr.grad), "r", rel_err(O.to_nchw_grad(rn).cpu(), rr.grad))
    for i in range(4):
        print("w", i, rel_err(wd[i].grad.cpu(), wr[i].grad), "b", rel_err(bd[i].grad.cpu(), br[i].grad))


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:7]])
