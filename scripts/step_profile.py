"""A clean train-step workload for rocprofv3: the C2 step (bs16 256x256) captured as a HIP graph and replayed
``--steps`` times, fp32 or under AMP (``--amp``).  Used by scripts/profile_round.sh for per-kernel stats.

    rocprofv3 --kernel-trace --stats -d out -- python3 scripts/step_profile.py [--amp] [--steps 10]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"), REPO]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--amp", action="store_true")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--eval", action="store_true", help="eval forward (encode+decode) instead of a train step")
    ap.add_argument("--serial", action="store_true", help="branch streams off (every kernel on the main stream)")
    ap.add_argument("--marker", action="store_true",
                    help="a torch spin kernel between the warm-up and the timed steps (scripts/step_traffic.py)")
    args = ap.parse_args()
    from hyres_hip.graphs import CapturedStep
    from hyres_hip.loss import RateDistortionLoss
    from hyres_hip import ops as O
    if args.serial:
        O.BranchStreams.enabled = False
    from hyres_hip.optim import DeviceGradScaler, FusedAdam
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    dev = torch.device("cuda:0")
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).train()
    g = torch.Generator().manual_seed(1926)
    x_cpu = torch.randint(0, 256, (args.batch, 3, args.size, args.size), generator=g).float() / 255
    jpeg, bpp = net.jpeg(x_cpu)
    x, jpeg = x_cpu.to(dev), jpeg.to(dev)
    main_p = [p for n, p in sorted(net.named_parameters()) if not n.endswith(".quantiles")]
    aux_p = [p for n, p in sorted(net.named_parameters()) if n.endswith(".quantiles")]
    opt = FusedAdam(main_p, lr=3e-4, max_grad_norm=1.0)
    aux_opt = FusedAdam(aux_p, lr=3e-4)
    crit = RateDistortionLoss(lmbda=0.045, alpha=0)
    if args.eval:
        net.eval()
        cap = CapturedStep(net, x, jpeg, bpp, amp=args.amp)
        step = cap.replay
    else:
        scaler = DeviceGradScaler(dev) if args.amp else None
        cap = CapturedStep(net, x, jpeg, bpp, criterion=crit, zero_grad=opt.zero_grad, amp=args.amp,
                           loss_scale=None if scaler is None else scaler.scale)

        def step():
            cap.replay()
            if scaler is not None:
                opt.step(grad_scaler=scaler)
                scaler.update(opt.sumsq)
            else:
                opt.step()
            opt.zero_grad()
            aux = net.aux_loss()
            aux.backward()
            aux_opt.step()
            aux_opt.zero_grad()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    if args.marker:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    print(f"{'eval' if args.eval else 'train'} {'amp' if args.amp else 'fp32'}: "
          f"{(time.time() - t0) * 1000 / args.steps:.3f} ms/step")


if __name__ == "__main__":
    main()
