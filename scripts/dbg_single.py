"""Debug: one conv layer (tape forward + backward) vs torch CPU at a given geometry; prints each error."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"), os.path.join(REPO, "tests")]
import torch
import torch.nn.functional as F
from helpers import rel_err


def run(B, H, W, Ci, Co, K):
    from hyres_hip import ops as O
    g = torch.Generator().manual_seed(1)
    x = torch.rand((B, Ci, H, W), generator=g) * 2 - 1
    w = (torch.rand((Co, Ci, K, K), generator=g) * 2 - 1) / (Ci * K * K) ** 0.5
    b = torch.rand((Co,), generator=g) * 0.2 - 0.1
    xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    yr = F.conv2d(xr, wr, br, padding=K // 2)
    gy = torch.rand(yr.shape, generator=g) * 2 - 1
    yr.backward(gy)
    D = torch.device("cuda:0")
    wd, bd = torch.nn.Parameter(w.to(D)), torch.nn.Parameter(b.to(D))
    tape = O.Tape()
    xn = O.to_nhwc(x.to(D), rg=True)
    yn = O.conv2d(tape, xn, wd, bd, pad=K // 2)
    yn.set_grad(O.nchw_grad_to_nhwc(gy.to(D)))
    tape.backward()
    torch.cuda.synchronize()
    print(B, H, W, Ci, Co, K, "y", rel_err(O.to_nchw(yn).cpu(), yr), "dx", rel_err(O.to_nchw_grad(xn).cpu(), xr.grad),
          "dw", rel_err(wd.grad.cpu(), wr.grad), "db", rel_err(bd.grad.cpu(), br.grad))


if __name__ == "__main__":
    for shp in ((1, 183, 183, 64, 128, 1), (1, 183, 183, 128, 64, 1), (1, 182, 182, 64, 128, 1), (1, 183, 183, 64, 64, 1),
                (1, 183, 183, 64, 128, 3), (1, 183, 183, 128, 128, 1), (1, 181, 181, 64, 128, 1), (1, 101, 101, 64, 128, 1)):
        run(*shp)
