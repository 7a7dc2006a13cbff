"""Peak device memory of the C2 train step (bs16 256x256), eager and graph-captured, fp32 and AMP: one line per
mode. Run twice — with HYRES_WGRAD_DEFER=1 (default) and =0 — to price the deferred split-K reduces' slabs
(hyres_hip.ops.WgradBatch keeps them alive until its flush).

    python3 scripts/mem_probe.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"), REPO]

import torch  # noqa: E402


def main():
    from hyres_hip.graphs import CapturedStep
    from hyres_hip.loss import RateDistortionLoss
    from hyres_hip.optim import FusedAdam
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    dev = torch.device("cuda:0")
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).train()
    g = torch.Generator().manual_seed(1926)
    x_cpu = torch.randint(0, 256, (16, 3, 256, 256), generator=g).float() / 255
    jpeg, bpp = net.jpeg(x_cpu)
    x, jpeg = x_cpu.to(dev), jpeg.to(dev)
    opt = FusedAdam([p for n, p in sorted(net.named_parameters()) if not n.endswith(".quantiles")], lr=3e-4)
    crit = RateDistortionLoss(lmbda=0.045, alpha=0)
    defer = os.environ.get("HYRES_WGRAD_DEFER", "1")
    for amp in (False, True):
        ctx = torch.autocast("cuda", dtype=torch.float16) if amp else torch.autocast("cuda", enabled=False)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        for _ in range(2):
            with ctx:
                out = net.forward_device(x, jpeg, bpp, noisequant=False)
                c = crit(out, x)
            c["loss"].backward()
            opt.zero_grad()
            del out, c
        torch.cuda.synchronize()
        eager_peak = torch.cuda.max_memory_allocated() - base
        torch.cuda.reset_peak_memory_stats()
        cap = CapturedStep(net, x, jpeg, bpp, criterion=crit, zero_grad=opt.zero_grad, amp=amp)
        cap.replay()
        torch.cuda.synchronize()
        graph_peak = torch.cuda.max_memory_allocated() - base
        cap.close()
        del cap
        print(f"WGRAD_DEFER={defer} {'amp' if amp else 'fp32'}: eager step peak {eager_peak / 2**30:.3f} GiB, "
              f"capture+replay peak {graph_peak / 2**30:.3f} GiB", flush=True)


if __name__ == "__main__":
    main()
