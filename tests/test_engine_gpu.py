"""The drop-in training loop (src/utils/engine.py train_one_epoch, the train.sh path) with its forward +
loss + backward replayed as HIP graphs equals the same loop run eagerly (HYRES_TRAIN_GRAPH=0), in fp32
and under --mixed-precision, with and without gradient accumulation (reference: src/utils/engine.py:8-90).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Images(torch.utils.data.Dataset):
    def __init__(self, n, size, seed):
        g = torch.Generator().manual_seed(seed)
        base = torch.nn.functional.interpolate(torch.rand(n, 3, size // 8, size // 8, generator=g), size=(size, size),
                                               mode="bilinear", align_corners=False)
        self.x = ((0.8 * base + 0.2 * torch.rand(n, 3, size, size, generator=g)) * 255).floor() / 255

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i]


def _train(graph, amp, accum, monkeypatch):
    from models import ResidualJPEGCompression
    from hyres_hip.weights import synthetic_state_dict
    from hyres_hip.loss import RateDistortionLoss
    from hyres_hip.optim import FusedAdam
    from src.utils.engine import train_one_epoch
    monkeypatch.setenv("HYRES_TRAIN_GRAPH", "1" if graph else "0")
    dev = torch.device("cuda:0")
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(dev)
    # the EntropyBottleneck / GaussianConditional training noise is drawn from host seeds in an eager step
    # and from a device-resident seed inside a graph (statistically the same, not the same numbers):
    # inject fixed draws so the two loops are comparable element by element
    g = torch.Generator().manual_seed(3)
    net.residual_model.noise.injected = {
        "z": (torch.rand(2, 2, 2, 128, generator=g) - 0.5).to(dev),
        "y": (torch.rand(2, 8, 8, 192, generator=g) - 0.5).to(dev)}
    named = sorted(net.named_parameters())
    opt = FusedAdam([p for n, p in named if not n.endswith(".quantiles")], lr=1e-4, max_grad_norm=1.0)
    aux = FusedAdam([p for n, p in named if n.endswith(".quantiles")], lr=1e-3)
    loader = torch.utils.data.DataLoader(_Images(8, 64, 5), batch_size=2, shuffle=False)
    crit = RateDistortionLoss(lmbda=0.045, alpha=0)
    loss, bpp, mse = train_one_epoch(net, crit, loader, opt, aux, 0, 1.0, noisequant=False, mixed_precision=amp,
                                     gradient_accumulation_steps=accum)
    torch.cuda.synchronize()
    return {n: p.detach().clone() for n, p in net.named_parameters()}, (loss, bpp, mse)


@pytest.mark.parametrize("amp,accum", [(False, 1), (False, 2), (True, 2)])
def test_graphed_training_loop_matches_eager(amp, accum, monkeypatch):
    pg, mg = _train(True, amp, accum, monkeypatch)
    pe, me = _train(False, amp, accum, monkeypatch)
    for a, b in zip(mg, me):
        assert abs(a - b) <= 1e-6 * max(abs(b), 1.0), (mg, me)
    worst = max(float((pg[n] - pe[n]).abs().max() / pe[n].abs().max().clamp_min(1e-12)) for n in pe)
    assert worst <= 1e-6, worst
    # the loop really trained (parameters moved from the synthetic initialisation)
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    init = synthetic_state_dict(ResidualJPEGCompression(jpeg_quality=50).state_dict())
    assert any(not torch.equal(pe[n].cpu(), init[n]) for n in pe)
