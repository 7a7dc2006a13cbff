"""Training CLI (src/training.py:28-312) — same flags as the reference, HIP hot path underneath.

Single GPU:   python -m src.training -d ./data --N 128 --M 192 ... (train.sh flags)
Multi-GPU:    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m src.training -d ./data ...
              (one process per GPU; batch-size is per rank; RCCL gradient all-reduce; rank 0 saves)
"""
import argparse
import os
import random
import sys
import warnings

import torch
from torch.utils.data import DataLoader

from models import LightWeightCheckerboard, ResidualJPEGCompression

from .losses import RateDistortionLoss
from .utils import DelfileList, ImageFolder, configure_optimizers, save_checkpoint, test_epoch, train_one_epoch
from .utils import transforms


def parse_args(argv):
    p = argparse.ArgumentParser(description="Example training script.")
    p.add_argument("-d", "--dataset", type=str, required=True, help="Training dataset")
    p.add_argument("--N", default=128, type=int, help="Number of channels of main codec")
    p.add_argument("--M", default=192, type=int, help="Number of channels of latent")
    p.add_argument("--jpeg-quality", default=1, type=int, help="JPEG quality factor (default: %(default)s)")
    p.add_argument("-e", "--epochs", default=4000, type=int, help="Number of epochs (default: %(default)s)")
    p.add_argument("-lr", "--learning-rate", default=1e-4, type=float, help="Learning rate (default: %(default)s)")
    p.add_argument("-n", "--num-workers", type=int, default=4, help="Dataloaders threads (default: %(default)s)")
    p.add_argument("--lambda", dest="lmbda", type=float, default=15e-3,
                   help="Bit-rate distortion parameter (default: %(default)s)")
    p.add_argument("--alpha", dest="alpha", type=float, default=0.001,
                   help="Perceptual level parameter (VGG loss) (default: %(default)s)")
    p.add_argument("--batch-size", type=int, default=16, help="Batch size (default: %(default)s)")
    p.add_argument("--test-batch-size", type=int, default=32, help="Test batch size (default: %(default)s)")
    p.add_argument("--aux-learning-rate", type=float, default=1e-3,
                   help="Auxiliary loss learning rate (default: %(default)s)")
    p.add_argument("--patch-size", type=int, nargs=2, default=(256, 256),
                   help="Size of the patches to be cropped (default: %(default)s)")
    p.add_argument("--cuda", type=lambda x: str(x).lower() == "true", default=True,
                   help="Use cuda (default: %(default)s)")
    p.add_argument("--save", action="store_true", default=True, help="Save model to disk")
    p.add_argument("--seed", default=1926, type=float, help="Set random seed for reproducibility")
    p.add_argument("--clip_max_norm", default=1.0, type=float, help="gradient clipping max norm (default: %(default)s")
    p.add_argument("--pretrained", action="store_true", help="use the pretrain model to refine the models")
    p.add_argument("--mixed-precision", action="store_true", help="Use mixed precision training")
    p.add_argument("--gradient-accumulation-steps", type=int, default=1,
                   help="Number of updates steps to accumulate before performing a backward/update pass")
    p.add_argument("--gpu-id", default="0", type=str, help="id(s) for CUDA_VISIBLE_DEVICES")
    p.add_argument("--savepath", default="./checkpoint", type=str, help="Path to save the checkpoint")
    p.add_argument("--checkpoint", type=str, help="Path to a checkpoint")
    return p.parse_args(argv)


class _NullWriter:
    def add_scalar(self, *a, **k):
        pass


def main(argv):
    args = parse_args(argv)
    if args.alpha != 0:
        # RateDistortionLoss's VGG16 term (src/losses/vgg16.py) needs torchvision's ImageNet weights, which
        # cannot be downloaded here: fail before any data is touched unless a local copy is configured
        from hyres_hip.vgg import _default_weights_path
        if _default_weights_path() is None:
            raise SystemExit(f"--alpha {args.alpha}: the VGG perceptual term needs VGG16 ImageNet weights; set "
                             f"HYRES_VGG16_WEIGHTS to a local vgg16-397923af.pth (or pass --alpha 0, as train.sh does)")
    # host JPEG worker processes, spawned before this process touches the GPU (hyres_hip.jpeg_host)
    from hyres_hip import jpeg_host
    jpeg_host.start()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and "CUDA_VISIBLE_DEVICES" not in os.environ:
        os.environ["CUDA_VISIBLE_DEVICES"] = args.gpu_id
    if args.seed is not None:
        torch.manual_seed(int(args.seed) + rank)
        random.seed(int(args.seed) + rank)
    reducer = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        from src.utils.engine import host_group
        host_group()  # the per-step host agreement group, created once per run (not once per epoch)
    device = torch.device("cuda", local if world > 1 else 0)

    train_tf = transforms.Compose([transforms.RandomCrop(args.patch_size), transforms.ToTensor()])
    test_tf = transforms.Compose([transforms.CenterCrop(args.patch_size), transforms.ToTensor()])
    train_dataset = ImageFolder(args.dataset, split="train", transform=train_tf)
    test_dataset = ImageFolder(args.dataset, split="test", transform=test_tf)
    sampler = None
    if world > 1:
        from torch.utils.data.distributed import DistributedSampler
        sampler = DistributedSampler(train_dataset, num_replicas=world, rank=rank, shuffle=True)
    train_loader = DataLoader(train_dataset, batch_size=args.batch_size, num_workers=args.num_workers,
                              shuffle=sampler is None, sampler=sampler, pin_memory=False)
    # DDP: rank r evaluates test images r, r + world, ... (no padding duplicates); test_epoch all-reduces the meters
    test_shard = list(range(rank, len(test_dataset), world)) if world > 1 else None
    test_loader = DataLoader(test_dataset, batch_size=args.test_batch_size, num_workers=args.num_workers,
                             shuffle=False, sampler=test_shard, pin_memory=False)
    # rank 0's best-checkpoint image dump walks the WHOLE test set alone (the reference's first test images and
    # metrics), with no collective: the other ranks are already in the next epoch
    full_test_loader = test_loader if world == 1 else DataLoader(
        test_dataset, batch_size=args.test_batch_size, num_workers=args.num_workers, shuffle=False, pin_memory=False)

    net = ResidualJPEGCompression(base_model=LightWeightCheckerboard(N=args.N, M=args.M),
                                  jpeg_quality=args.jpeg_quality).to(device)
    if world > 1:
        from hyres_hip.ddp import broadcast_parameters
        broadcast_parameters(net)
    os.makedirs(args.savepath, exist_ok=True)
    try:
        from tensorboardX import SummaryWriter  # noqa: F401
        writer = SummaryWriter(args.savepath) if rank == 0 else _NullWriter()
    except Exception:  # noqa: BLE001 - tensorboardX is optional
        writer = _NullWriter()

    optimizer, aux_optimizer = configure_optimizers(net, args, max_grad_norm=args.clip_max_norm)
    if world > 1:
        from hyres_hip.ddp import FlatGradReducer, HYRES_SEGMENTS
        names = sorted(n for n, p in net.named_parameters() if not n.endswith(".quantiles") and p.requires_grad)
        reducer = FlatGradReducer(optimizer.flat, world, names=names, segments=HYRES_SEGMENTS).overlap()
    lr_scheduler = torch.optim.lr_scheduler.MultiStepLR(optimizer, milestones=[400], gamma=0.1)
    criterion = RateDistortionLoss(lmbda=args.lmbda, alpha=args.alpha)

    last_epoch = 0
    if args.checkpoint:
        print("Loading", args.checkpoint)
        ckpt = torch.load(args.checkpoint, map_location=device, weights_only=True)
        net.load_state_dict(ckpt["state_dict"])
        last_epoch = ckpt["epoch"] + 1
        optimizer.load_state_dict(ckpt["optimizer"])
        aux_optimizer.load_state_dict(ckpt["aux_optimizer"])
        lr_scheduler.load_state_dict(ckpt["lr_scheduler"])
    stemode = False
    if args.checkpoint and args.pretrained:
        stemode = True
        last_epoch = 0
        optimizer.param_groups[0]["lr"] = args.learning_rate
        aux_optimizer.param_groups[0]["lr"] = args.aux_learning_rate
        lr_scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, "min", factor=0.1, patience=10)

    noisequant = True
    best_loss = float("inf")
    for epoch in range(last_epoch, args.epochs):
        if sampler is not None:
            sampler.set_epoch(epoch)
        if epoch > 400 or stemode:
            noisequant = False
        if rank == 0:
            print(f"noisequant: {noisequant}, stemode:{stemode}")
            print(f"Learning rate: {optimizer.param_groups[0]['lr']}")
        train_loss, train_bpp, train_mse = train_one_epoch(
            net, criterion, train_loader, optimizer, aux_optimizer, epoch, args.clip_max_norm, noisequant,
            args.mixed_precision, args.gradient_accumulation_steps, reducer=reducer)
        writer.add_scalar("Train/loss", train_loss, epoch)
        writer.add_scalar("Train/mse", train_mse, epoch)
        writer.add_scalar("Train/bpp", train_bpp, epoch)
        loss, bpp, mse = test_epoch(epoch, test_loader, net, criterion)
        writer.add_scalar("Test/loss", loss, epoch)
        writer.add_scalar("Test/mse", mse, epoch)
        writer.add_scalar("Test/bpp", bpp, epoch)
        # src/training.py:265 calls lr_scheduler.step(loss) for BOTH schedulers; on MultiStepLR that is the
        # deprecated step(epoch=loss) whose closed form gives lr = base * 0.1 ** bisect([400], loss): with a
        # loss of O(1) the learning rate never decays.  Mirrored (drop-in training schedule), not fixed.
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", UserWarning)
            lr_scheduler.step(loss)
        is_best = loss < best_loss
        if args.save and rank == 0:
            state = {"epoch": epoch, "state_dict": net.state_dict(), "loss": loss,
                     "optimizer": optimizer.state_dict(), "aux_optimizer": aux_optimizer.state_dict(),
                     "lr_scheduler": lr_scheduler.state_dict()}
            DelfileList(args.savepath, "checkpoint_last")
            save_checkpoint(state, filename=os.path.join(args.savepath, f"checkpoint_last_{epoch}.pth.tar"))
            if is_best:
                best_loss = loss
                test_epoch(epoch, full_test_loader, net, criterion, save_images=True, savepath=args.savepath,
                           all_reduce=False)
                DelfileList(args.savepath, "checkpoint_best")
                save_checkpoint(state, filename=os.path.join(args.savepath, f"checkpoint_best_loss_{epoch}.pth.tar"))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1:])
