"""Worker for tests/test_ddp_gpu.py: the HIP-path data-parallel step (configs[3] / SURVEY §8e, replacing the
reference's nn.DataParallel, src/training.py:211-212) on WORLD_SIZE ranks that share device 0 over gloo
(RCCL refuses two ranks on one device; gloo all-reduces CUDA tensors through the host with the same stream
ordering, so the after-replay reduction runs unchanged).

Launched by ``python -m torch.distributed.run --nproc-per-node 2 … tests/ddp_world2_worker.py OUT``, before
the launching test touches anything but its own process.  Each rank:
  1. captures the train step (forward + RD loss + tape backward) as a HIP graph (``CapturedStep``);
  2. replays it on its half of a bs=4 64² batch (STE quantisation, injected EntropyBottleneck noise) and
     all-reduces the flat gradient after the replay (``FlatGradReducer.all_reduce``, bench.py's N > 1 mode);
  3. replays and reduces again: must equal (2) bit for bit (run-to-run determinism of the DDP step);
  4. takes one FusedAdam(clip 1.0) step; rank 0 then broadcasts its parameters, every rank checks equality;
Rank 0 finally re-runs each rank's shard single-process (their mean must equal the reduced gradient bit for
bit) and the whole bs=4 batch (fresh models, same weights), and saves the flat gradients + losses to OUT.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"))
sys.path.insert(0, REPO)


def batch(n=4, size=64, seed=11):
    g = torch.Generator().manual_seed(seed)
    base = torch.nn.functional.interpolate(torch.rand(n, 3, size // 8, size // 8, generator=g), size=(size, size),
                                           mode="bilinear", align_corners=False)
    x = ((0.8 * base + 0.2 * torch.rand(n, 3, size, size, generator=g)) * 255).floor() / 255
    nz = torch.rand(n, size // 32, size // 32, 128, generator=g) - 0.5
    ny = torch.rand(n, size // 8, size // 8, 192, generator=g) - 0.5
    return x, nz, ny


def build(dev):
    from models import ResidualJPEGCompression
    from hyres_hip.weights import synthetic_state_dict
    from hyres_hip.optim import FusedAdam
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).train()
    named = sorted(net.named_parameters())
    names = [n for n, _ in named if not n.endswith(".quantiles")]
    opt = FusedAdam([p for n, p in named if not n.endswith(".quantiles")], lr=1e-4, max_grad_norm=1.0)
    return net, names, opt


def main():
    out_path = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    from hyres_hip.ddp import FlatGradReducer, HYRES_SEGMENTS, broadcast_parameters
    from hyres_hip.graphs import CapturedStep
    from hyres_hip.loss import RateDistortionLoss

    x_all, nz_all, ny_all = batch()
    per = x_all.shape[0] // world
    sl = slice(rank * per, (rank + 1) * per)
    net, names, opt = build(dev)
    broadcast_parameters(net)
    crit = RateDistortionLoss(lmbda=0.045, alpha=0)
    jd, bpp = net.jpeg(x_all[sl])
    x, j = x_all[sl].to(dev), jd.to(dev)
    net.residual_model.noise.injected = {"z": nz_all[sl].to(dev), "y": ny_all[sl].to(dev)}

    red = FlatGradReducer(opt.flat, world, names=names, segments=HYRES_SEGMENTS)
    # HYRES_DDP_SPLIT=1: bench.py's graph+overlap mode — the capture cut at the "hyper" marker, the finished segments'
    # all-reduce started between the two replays (while g_a's backward replays), the rest after
    split = os.environ.get("HYRES_DDP_SPLIT", "0") == "1"
    cap = CapturedStep(net, x, j, float(bpp), criterion=crit, zero_grad=opt.zero_grad,
                       capture_error_mode="thread_local", split_at=("hyper",) if split else ())
    between = red.launch_segments if split else None
    if split:
        assert len(cap.graphs) == 2 and cap.segments_done == [["refine", "g_s", "hyper"]], cap.segments_done

    opt.zero_grad()
    c = cap.replay(between=between)[1]
    red.all_reduce()
    torch.cuda.synchronize()
    g_ddp = opt.flat.grad.clone()
    loss = c["loss"].detach().clone()
    dist.all_reduce(loss)
    loss_mean = float(loss) / world

    opt.zero_grad()
    cap.replay(between=between)
    red.all_reduce()
    torch.cuda.synchronize()
    same_after = bool(torch.equal(opt.flat.grad, g_ddp))
    c = None
    cap.close()

    opt.step()
    torch.cuda.synchronize()
    mine = opt.flat.data.clone()
    ref = opt.flat.data.clone()
    dist.broadcast(ref, src=0)
    params_equal = torch.zeros(1, device=dev)
    params_equal += float(torch.equal(mine, ref))
    dist.all_reduce(params_equal)
    params_equal_all = int(params_equal) == world

    if rank == 0:
        def single(sl_):
            """The same graphed step in one process on the batch slice ``sl_`` (fresh model, same weights)."""
            net1, _, opt1 = build(dev)
            jd1, bpp1 = net1.jpeg(x_all[sl_])
            net1.residual_model.noise.injected = {"z": nz_all[sl_].to(dev), "y": ny_all[sl_].to(dev)}
            cap1 = CapturedStep(net1, x_all[sl_].to(dev), jd1.to(dev), float(bpp1), criterion=crit,
                                zero_grad=opt1.zero_grad)
            opt1.zero_grad()
            c1 = cap1.replay()[1]
            torch.cuda.synchronize()
            return opt1.flat.grad.clone(), float(c1["loss"])

        # (a) each rank's shard recomputed here: their mean is what the all-reduce must produce, bit for bit
        # (sum of two fp32 values, then x 1/world — the reducer's exact arithmetic)
        halves = [single(slice(r * per, (r + 1) * per)) for r in range(world)]
        g_mean = halves[0][0]
        for gh, _ in halves[1:]:
            g_mean = g_mean + gh
        g_mean = g_mean * (1.0 / world)
        # (b) the whole batch in one process: equal up to batch-size-dependent summation order
        g_all, loss_all = single(slice(0, x_all.shape[0]))
        offs = np.array(opt.flat.offsets, dtype=np.int64)
        sizes = np.array([p.numel() for p in opt.flat.params], dtype=np.int64)
        np.savez(out_path, g_ddp=g_ddp.cpu().numpy(), g_mean=g_mean.cpu().numpy(),
                 g_single=g_all.cpu().numpy(), loss_ddp=np.float64(loss_mean), loss_single=np.float64(loss_all),
                 same_after=np.bool_(same_after), params_equal=np.bool_(params_equal_all),
                 offsets=offs, sizes=sizes, names=np.array(names))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
