"""CPU, world_size 2 over gloo: the data-parallel gradient path (hyres_hip/ddp.py) that replaces the
reference's nn.DataParallel (src/training.py:211-212, src/utils/dataset_utils.py:76-82).

* FlatGradReducer averages the flat gradient buffer across ranks bucket by bucket (odd sizes, bucket
  boundaries inside parameters);
* broadcast_parameters makes every rank start from rank 0's weights;
* the semantic claim of SURVEY.md §8(e): with equal shards, averaging the per-rank gradients of the
  per-rank RD loss (src/losses/rd_loss.py:18-44 normalises by the LOCAL N*H*W) equals the gradient of
  the global-batch loss.  Checked with the oracle on the committed reference fixture batch (2 images,
  one per rank).
"""
import os
import socket
import sys
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _reducer_worker(rank, world, port):
    _init(rank, world, port)
    try:
        from hyres_hip.ddp import FlatGradReducer, broadcast_parameters
        from hyres_hip.optim import FlatParams
        shapes = [(7,), (3, 5), (129,), (2, 2, 3), (1,), (64, 3)]
        gen = torch.Generator().manual_seed(100 + rank)  # ranks start from different weights
        params = [torch.nn.Parameter(torch.randn(s, generator=gen)) for s in shapes]
        mod = torch.nn.Module()
        for i, p in enumerate(params):
            mod.register_parameter(f"p{i}", p)
        mod.register_buffer("buf", torch.full((5,), float(rank)))
        broadcast_parameters(mod)
        g0 = torch.Generator().manual_seed(100)
        ref = [torch.randn(s, generator=g0) for s in shapes]
        for p, r in zip(params, ref):
            assert torch.equal(p.data, r)
        assert torch.equal(mod.buf, torch.zeros(5))
        flat = FlatParams(params)
        for i, p in enumerate(params):
            p.grad.copy_(torch.arange(p.numel(), dtype=torch.float32).view_as(p) * (rank + 1) + i)
        red = FlatGradReducer(flat, world, bucket_bytes=40)  # 10 floats per bucket: boundaries inside params
        assert len(red.buckets) > len(params)
        red.all_reduce()
        mean_scale = sum(r + 1 for r in range(world)) / world
        for i, p in enumerate(params):
            want = torch.arange(p.numel(), dtype=torch.float32).view_as(p) * mean_scale + i
            assert torch.allclose(p.grad, want, rtol=0, atol=1e-6), i
        # params are views of the flat buffer; the 16-byte alignment padding stays zero
        for p, o in zip(params, flat.offsets):
            assert p.data.data_ptr() == flat.data.data_ptr() + 4 * o
    finally:
        dist.destroy_process_group()


def _grad_vector(orc_sd, keys):
    out = []
    for k in keys:
        t = orc_sd[k]
        out.append(torch.zeros(t.numel()) if t.grad is None else t.grad.detach().reshape(-1).clone())
    return torch.cat(out)


def _oracle_grads(x, jpeg, lmbda, jpeg_bpp):
    from helpers import oracle_from, recipe_state_dict, _is_param_key
    from oracle import rd_loss
    sd = recipe_state_dict()
    orc, sd2 = oracle_from(sd, requires_grad=True)
    out = orc.forward(x, jpeg, jpeg_bpp, training=False)
    out["jpeg_bpp_loss"] = torch.tensor(jpeg_bpp)
    rd_loss(out, x, lmbda)["loss"].backward()
    keys = [k for k in sd2 if _is_param_key(k) and sd2[k].is_floating_point() and sd2[k].requires_grad]
    return _grad_vector(sd2, keys), keys


def _sharded_worker(rank, world, port):
    _init(rank, world, port)
    try:
        sys.path.insert(0, HERE)
        from helpers import load_meta, load_npz
        from hyres_hip.ddp import FlatGradReducer
        g = load_npz("hyres_eval_b2_64.npz")
        meta = load_meta()
        lmbda = meta["train_lambda"]
        jb = float(g["jpeg_bpp"])
        x, jpeg = g["x"], g["jpeg_decoded"]
        assert x.shape[0] == world
        vec, keys = _oracle_grads(x[rank:rank + 1], jpeg[rank:rank + 1], lmbda, jb)
        flat = types.SimpleNamespace(grad=vec, numel=vec.numel())
        FlatGradReducer(flat, world, bucket_bytes=1 << 20).all_reduce()
        if rank == 0:
            full, _ = _oracle_grads(x, jpeg, lmbda, jb)
            err = float((vec - full).norm() / full.norm())
            assert err < 1e-5, err
    finally:
        dist.destroy_process_group()


def test_flat_grad_reducer_gloo_world2():
    mp.spawn(_reducer_worker, args=(2, _free_port()), nprocs=2, join=True)


def test_sharded_gradient_equals_global_batch_gloo_world2():
    mp.spawn(_sharded_worker, args=(2, _free_port()), nprocs=2, join=True)


def _overlap_worker(rank, world, port):
    """Segmented all-reduce launched from backward-progress markers (hyres_hip.ops.GradReady) during the
    tape backward, the remainder after it: same mean as the plain bucketed reduce; not armed (gradient
    accumulation micro-batch) -> markers launch nothing."""
    _init(rank, world, port)
    try:
        from hyres_hip.ddp import FlatGradReducer, HYRES_SEGMENTS
        from hyres_hip.ops import GradReady, Tape
        from hyres_hip.optim import FlatParams
        names = sorted(["refine.conv.weight", "refine.conv.bias", "residual_model.g_a.0.weight",
                        "residual_model.g_s.0.weight", "residual_model.h_a.0.weight",
                        "residual_model.param_aggregation.0.bias", "residual_model.g_s.1.beta"])
        shapes = [(5, 3), (3,), (4, 4), (7,), (2, 9), (6,), (11,)]
        params = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
        flat = FlatParams(params)
        red = FlatGradReducer(flat, world, bucket_bytes=24, names=names, segments=HYRES_SEGMENTS)
        assert set(red.segments) == {"refine", "g_s", "hyper"}
        GradReady.listeners = []
        red.overlap()
        fired = []
        for armed in (True, False):
            flat.grad.zero_()
            red.armed = armed
            tape = Tape()
            # forward order: g_a, [hyper mark], h_a/param_agg, [g_s mark], g_s, [refine mark], refine
            owner = {"hyper": ("residual_model.h_a.", "residual_model.param_aggregation."),
                     "g_s": ("residual_model.g_s.",), "refine": ("refine.",)}

            def writer(prefixes):
                def w():
                    for i, (n, p) in enumerate(zip(names, params)):
                        if n.startswith(prefixes):
                            p.grad.copy_(torch.full(p.shape, float((rank + 1) * (i + 1))))
                return w

            tape.push(writer(("residual_model.g_a.",)))
            for mk in ("hyper", "g_s", "refine"):
                GradReady.mark(tape, mk)
                tape.push(writer(owner[mk]))
            tape.backward()
            fired.append(list(red.fired))
            if not armed:
                assert red.fired == [] and red.works == []
                continue
            assert red.fired == ["refine", "g_s", "hyper"] and len(red.works) > 0
            red.all_reduce()
            mean = sum(r + 1 for r in range(world)) / world
            for i, p in enumerate(params):
                assert torch.allclose(p.grad, torch.full(p.shape, mean * (i + 1))), names[i]
        GradReady.listeners = []
    finally:
        dist.destroy_process_group()


def test_overlapped_segment_reduce_gloo_world2():
    mp.spawn(_overlap_worker, args=(2, _free_port()), nprocs=2, join=True)


def _engine_host_worker(rank, world, port):
    """src/utils/engine.py's host-side DDP pieces: the sharded test epoch's meter all-reduce and the per-step
    capture-key agreement (a rank at a different batch shape raises instead of hanging)."""
    _init(rank, world, port)
    try:
        from src.losses import AverageMeter
        from src.utils.engine import _GraphedStep, _all_reduce_meters, _all_ranks_ok, host_group
        m = AverageMeter()
        for v in ([1.0, 2.0] if rank == 0 else [4.0]):  # ragged shards: 2 batches on rank 0, 1 on rank 1
            m.update(v)
        _all_reduce_meters([m], "cpu")
        assert m.count == 3 and abs(m.avg - 7.0 / 3) < 1e-12
        gs = _GraphedStep.__new__(_GraphedStep)
        gs._host_group = host_group()
        assert gs._host_group is not None and host_group() is gs._host_group  # one group per run, not per epoch
        gs._agree(((16, 3, 256, 256), False, False))  # same key on both ranks: passes
        assert _all_ranks_ok(rank == 0, gs._host_group) is False  # one rank failed: every rank falls back
        assert _all_ranks_ok(True, gs._host_group) is True
        with pytest.raises(RuntimeError, match="different graph-capture keys"):
            gs._agree(((16 if rank == 0 else 12, 3, 256, 256), False, False))
    finally:
        dist.destroy_process_group()


def test_engine_ddp_host_agreement_gloo_world2():
    mp.spawn(_engine_host_worker, args=(2, _free_port()), nprocs=2, join=True)


class _FakeNet(torch.nn.Module):
    """Stands in for ResidualJPEGCompression in test_epoch (CPU): the output dict's image tensors and aux_loss."""

    def __init__(self):
        super().__init__()
        self.p = torch.nn.Parameter(torch.zeros(1))

    def forward(self, d):
        return {"x_hat": d.clamp(0, 1), "jpeg_decoded": d, "residual": d - 0.5, "residual_hat": d - 0.5}

    def aux_loss(self):
        return self.p.sum() + 1.0


def _fake_criterion(out, d):
    v = d.mean()
    return {k: v * (i + 1) for i, k in enumerate(("loss", "bpp_loss", "residual_bpp_loss", "y_bpp_loss",
                                                   "z_bpp_loss", "mse_loss"))}


def _save_epoch_worker(rank, world, port, savepath):
    """The best-checkpoint image dump (src/training.py: ``if args.save and rank == 0``) runs test_epoch on rank 0
    ALONE over the whole test set. It must issue no collective: rank 1 is already in the next epoch's all-reduce,
    and a meter all-reduce on rank 0 would pair with it (wrong sums or a hang)."""
    _init(rank, world, port)
    try:
        from src.utils.engine import test_epoch
        data = [torch.full((1, 3, 8, 8), 0.1 * (i + 1)) for i in range(4)]
        shard = data[rank::world]
        net = _FakeNet()
        loss, _, _ = test_epoch(0, shard, net, _fake_criterion)  # sharded epoch: meters summed over ranks
        assert abs(loss - sum(float(t.mean()) for t in data) / len(data)) < 1e-6
        if rank == 0:
            loss0, _, _ = test_epoch(0, data, net, _fake_criterion, save_images=True, savepath=savepath,
                                     all_reduce=False)
            assert abs(loss0 - loss) < 1e-6  # the whole test set on rank 0 alone
            assert os.path.exists(os.path.join(savepath, "best_metrics.csv"))
            assert os.path.exists(os.path.join(savepath, "best_recon", "recon_3.png"))
        nxt = torch.tensor([float(rank + 1)])  # "the next epoch's" collective
        dist.all_reduce(nxt)
        assert float(nxt) == 3.0
    finally:
        dist.destroy_process_group()


def test_best_checkpoint_save_epoch_gloo_world2(tmp_path):
    mp.spawn(_save_epoch_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
