"""fp32 GEMM on the bf16 MFMA ("bf16x6", hyres_conv_tuning key HYRES_TUNE_F32_GEMM = 7, csrc/conv.hip
conv3x3_wres_bf6_kernel): each fp32 operand is split into three bf16 pieces and each product formed from the six
cross products with i + j <= 2, fp32 accumulation. Claim under test: it is as accurate as the native fp32 MFMA
(v_mfma_f32_32x32x2_f32, an fmaf chain) — per product ~2^-25 relative against fp32's 2^-24 rounding — so the fp32
parity bars of the model hold unchanged. Checked against float64 on the 3x3 64->64 convs the kernel serves
(forward with bias / residual / ReLU) and on every implicit-GEMM tile family. bf16x6 is the default fp32 GEMM; the
fp32 parity suite (tests/test_parity_gpu.py: conv / deconv / GDN forward and backward, the masked conv, the model train
step against the reference fixture and the C2-size train step against the fp64 oracle) runs on both GEMMs through its
``fp32_gemm`` fixture."""
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


class _Bf6:
    def __init__(self, on):
        self.on = on

    def __enter__(self):
        import ctypes
        from hyres_hip import _lib as L
        self.old = ctypes.c_int(0)
        L.call("hyres_conv_tuning", 7, 1 if self.on else 0, ctypes.byref(self.old))
        return self

    def __exit__(self, *a):
        from hyres_hip import _lib as L
        L.call("hyres_conv_tuning", 7, self.old.value, None)


def test_bf6_conv3x3_as_accurate_as_fp32():
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    import ctypes
    D = dev()
    B, C, H, W = 4, 64, 128, 128  # 256 tiles: the weight-resident kernel's eligibility (2 tiles per block)
    x = _rand((B, C, H, W), 1).to(D)
    w = _rand((C, C, 3, 3), 2, (C * 9) ** -0.5).to(D)
    b = _rand((C,), 3, 0.1).to(D)
    r = _rand((B, C, H, W), 4).to(D)
    ref = F.relu(F.conv2d(x.double(), w.double(), b.double(), padding=1) + r.double())
    outs, names = {}, {}
    for on in (False, True):
        with _Bf6(on):
            xn, rn = O.to_nhwc(x), O.to_nhwc(r)
            g = O._geom("hyres_geom_conv2d", B, H, W, C, C, C, C, 3, 3, 1, 1, 1)
            e = L.Epilogue()
            e.kind, e.act, e.bias, e.res, e.ldres = L.EPI_BIAS, L.ACT_RELU, b.data_ptr(), rn.ptr(), C
            names[on] = O.conv_variant(g, e, False)
            yn = O.conv2d(None, xn, torch.nn.Parameter(w), b, pad=1, act=L.ACT_RELU, res=rn)
            outs[on] = O.to_nchw(yn).double()
    torch.cuda.synchronize()
    assert names[True] == "conv3x3_wres_bf6_kernel" and names[False] == "conv3x3_wres_f32_kernel", names
    e32, e6 = rel_err(outs[False].cpu(), ref.cpu()), rel_err(outs[True].cpu(), ref.cpu())
    d = (outs[True] - ref).abs().max().item(), (outs[False] - ref).abs().max().item()
    print(f"3x3 64->64 +res relu, max-norm error vs fp64: native fp32 {e32:.2e}, bf16x6 {e6:.2e} (abs {d})")
    assert e6 <= 2.0 * e32 + 1e-9 and e6 < 1e-6


@pytest.mark.parametrize("case", [
    # B, Ci, Co, H, K, stride, (the implicit-GEMM families of the fp32 step)
    (2, 128, 128, 64, 5, 2),   # g_a 5x5 stride 2 (128x128 tiles)
    (4, 64, 128, 64, 1, 1),    # short-K 1x1 (64x128 tiles)
    (16, 96, 96, 32, 3, 1),    # AttentionBlock(192) 3x3 at 32^2 (64x64 tiles, small grid)
    (2, 384, 192, 16, 3, 1),   # hyperprior 3x3 (split-K)
])
def test_bf6_implicit_gemm_conv_as_accurate_as_fp32(case):
    """conv_fwd_b6_kernel (hyres_conv_tuning key 7 on the implicit-GEMM conv): forward with bias, every tile family
    and split-K, against float64; error no worse than twice the native fp32 kernel's."""
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    B, Ci, Co, H, K, s = case
    D = dev()
    x = _rand((B, Ci, H, H), 21).to(D)
    w = _rand((Co, Ci, K, K), 22, (Ci * K * K) ** -0.5).to(D)
    b = _rand((Co,), 23, 0.1).to(D)
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=s, padding=K // 2)
    outs, names = {}, {}
    for on in (False, True):
        with _Bf6(on):
            xn = O.to_nhwc(x)
            yn = O.conv2d(None, xn, torch.nn.Parameter(w), b, stride=s, pad=K // 2)
            outs[on] = O.to_nchw(yn).double()
            g = O._geom("hyres_geom_conv2d", B, H, H, Ci, Ci, Co, Co, K, K, s, K // 2, 1)
            e = L.Epilogue()
            e.kind, e.bias = L.EPI_BIAS, b.data_ptr()
            names[on] = O.conv_variant(g, e, O.conv_split(g, e) > 1)
    torch.cuda.synchronize()
    e32, e6 = rel_err(outs[False].cpu(), ref.cpu()), rel_err(outs[True].cpu(), ref.cpu())
    print(case, names, f"error vs fp64: native {e32:.2e}, bf16x6 {e6:.2e}")
    assert names[True].startswith(("conv_fwd_b6_kernel", "conv_fwd_b6db_kernel", "conv3x3_wres_bf6")), names[True]
    assert e6 <= 2.0 * e32 + 1e-9 and e6 < 1e-5


@pytest.mark.parametrize("B,H,W,act", [(1, 256, 384, "relu"), (1, 512, 768, "prelu"), (2, 128, 192, "none")])
def test_bf6_conv3x3_wide_images(B, H, W, act):
    """The weight-resident 3x3 at the Kodak shapes (one 768x512 image: g_a / g_s at 384x256, MultiScaleRefine at full
    size with its PReLU), against float64: bf16x6 no worse than twice the native kernel."""
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    C = 64
    x = _rand((B, C, H, W), 31).to(D)
    w = _rand((C, C, 3, 3), 32, (C * 9) ** -0.5).to(D)
    b = _rand((C,), 33, 0.1).to(D)
    slope = torch.tensor([0.25], device=D)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1)
    if act == "relu":
        ref = F.relu(ref)
    elif act == "prelu":
        ref = torch.where(ref >= 0, ref, 0.25 * ref)
    a = {"relu": L.ACT_RELU, "prelu": L.ACT_PRELU, "none": L.ACT_NONE}[act]
    outs, names = {}, {}
    for on in (False, True):
        with _Bf6(on):
            xn = O.to_nhwc(x)
            g = O._geom("hyres_geom_conv2d", B, H, W, C, C, C, C, 3, 3, 1, 1, 1)
            e = L.Epilogue()
            e.kind, e.act, e.bias = L.EPI_BIAS, a, b.data_ptr()
            names[on] = O.conv_variant(g, e, False)
            yn = O.conv2d(None, xn, torch.nn.Parameter(w), b, pad=1, act=a, slope=slope if act == "prelu" else None)
            outs[on] = O.to_nchw(yn).double()
    torch.cuda.synchronize()
    e32, e6 = rel_err(outs[False].cpu(), ref.cpu()), rel_err(outs[True].cpu(), ref.cpu())
    print(B, H, W, act, names, f"error vs fp64: native {e32:.2e}, bf16x6 {e6:.2e}")
    assert e6 <= 2.0 * e32 + 1e-9 and e6 < 1e-5


@pytest.mark.parametrize("case", [
    # B, Ci (read), Ci_w (weight row), Co, H, W, K, ldy (output pixel stride)
    (1, 192, 192, 384, 64, 96, 3, 768),   # h_s's last conv into the [latent_params | context] buffer (split-K)
    (1, 384, 768, 640, 64, 96, 1, 640),   # param_aggregation.0, anchor pass: the first 384 of 768 input channels
    (1, 768, 768, 640, 64, 96, 1, 640),
    (1, 640, 640, 512, 64, 96, 1, 512),
])
def test_bf6_latent_layers_kodak(case):
    """The latent-resolution layers of one 768x512 image (64 x 96 latents: small grids, split-K, a strided output, a
    partial-channel read of the weight rows), bf16x6 against the native kernel and float64."""
    from hyres_hip import ops as O
    B, Ci, Ciw, Co, H, W, K, ldy = case
    D = dev()
    x = _rand((B, Ci, H, W), 41).to(D)
    w = _rand((Co, Ciw, K, K), 42, (Ci * K * K) ** -0.5).to(D)
    b = _rand((Co,), 43, 0.1).to(D)
    ref = F.conv2d(x.double(), w[:, :Ci].double(), b.double(), padding=K // 2)
    outs = {}
    for on in (False, True):
        with _Bf6(on):
            xn = O.to_nhwc(x)
            big = O.Node.new(B, H, W, ldy, D)
            yo = big.slice(0, Co)
            O.conv2d(None, xn, torch.nn.Parameter(w), b, pad=K // 2, out=yo)
            outs[on] = big.v[..., :Co].permute(0, 3, 1, 2).double()
    torch.cuda.synchronize()
    e32, e6 = rel_err(outs[False].cpu(), ref.cpu()), rel_err(outs[True].cpu(), ref.cpu())
    print(case, f"error vs fp64: native {e32:.2e}, bf16x6 {e6:.2e}")
    assert e6 <= 2.0 * e32 + 1e-9 and e6 < 1e-5


@pytest.mark.parametrize("garbage", [0.0, 1e3])
def test_bf6_partial_channel_read_of_strided_buffer(garbage):
    """param_aggregation.0 in the anchor pass exactly as the model runs it: the input is the first 2M = 384 channels of
    the [latent | ctx] NHWC buffer (pixel stride 768) whose ctx half is not yet written (filled here with 0 or with
    large values), the weight rows 768 wide; bf16x6 and native against float64 on the live half only."""
    from hyres_hip import ops as O
    D = dev()
    B, H, W, M2, Co = 1, 64, 96, 384, 640
    lat = _rand((B, M2, H, W), 51).to(D)
    w = _rand((Co, 2 * M2, 1, 1), 52, M2 ** -0.5).to(D)
    b = _rand((Co,), 53, 0.1).to(D)
    ref = F.conv2d(lat.double(), w[:, :M2].double(), b.double())
    outs = {}
    for on in (False, True):
        with _Bf6(on):
            lc = O.Node.new(B, H, W, 2 * M2, D)
            lc.v.fill_(garbage)
            lc.v[..., :M2] = lat.permute(0, 2, 3, 1)
            yn = O.conv2d(None, lc.slice(0, M2), torch.nn.Parameter(w), b)
            outs[on] = O.to_nchw(yn).double()
    torch.cuda.synchronize()
    e32, e6 = rel_err(outs[False].cpu(), ref.cpu()), rel_err(outs[True].cpu(), ref.cpu())
    print(f"garbage {garbage}: error vs fp64: native {e32:.2e}, bf16x6 {e6:.2e}")
    assert e32 < 1e-5 and e6 < 1e-5


def test_bf6_kodak_layers_match_native():
    """Layer by layer (every conv output with a fused ReLU / PReLU, in forward order, ops.Trace.acts) of the eval
    forward on one 768x512 image, bf16x6 against the native fp32 MFMA: g_a up to the latent y has no discontinuity
    (the first round() is after it), so every layer there must agree to fp32 noise (1e-5 max-norm relative); the
    first layers that differ more are printed with their shapes."""
    from hyres_hip import ops as O
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    D = dev()
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(D).eval()
    g = torch.Generator().manual_seed(7)
    base = F.interpolate(torch.rand(1, 3, 16, 24, generator=g), size=(512, 768), mode="bilinear", align_corners=False)
    x = ((base * 0.8 + 0.2 * torch.rand(1, 3, 512, 768, generator=g)) * 255).floor() / 255
    jpeg, jb = net.jpeg(x)
    runs = {}
    for on in (False, True):
        O.Trace.nodes, O.Trace.acts = {}, []
        with _Bf6(on), torch.no_grad():
            net(x, jpeg=(jpeg, jb))
        torch.cuda.synchronize()
        runs[on] = ([(tuple(n.v.shape), O.to_nchw(n).double().cpu()) for _, n, _ in O.Trace.acts],
                    {k: O.Trace.value(k).double().cpu() for k in O.Trace.nodes})
        O.Trace.nodes, O.Trace.acts = None, None
    a, b = runs[False][0], runs[True][0]
    assert len(a) == len(b)
    rows = [(i, a[i][0], rel_err(b[i][1], a[i][1])) for i in range(len(a))]
    bad = [r for r in rows if r[2] > 1e-5]
    print("layers beyond 1e-5 (index, NHWC shape, max-norm rel diff):", bad[:12])
    for k in runs[False][1]:
        print(f"stage {k}: {tuple(runs[False][1][k].shape)} bf16x6 vs native {rel_err(runs[True][1][k], runs[False][1][k]):.2e}")
    # the first diverging layer recomputed in float64 from its traced input, for both runs
    pa = net.residual_model.param_aggregation
    w0, b0 = pa[0].weight.detach().double().cpu(), pa[0].bias.detach().double().cpu()
    for on in (False, True):
        lat = runs[on][1]["latent_params"]
        want = F.relu(F.conv2d(lat, w0[:, :lat.shape[1]], b0))
        got = [t for shp, t in runs[on][0] if shp[-1] == 640]
        print(f"bf16x6={on}: param_aggregation.0 (anchor) vs float64 from the traced latent: "
              f"{rel_err(got[0], want):.2e}; non-anchor count {len(got)}")
    ey = rel_err(runs[True][1]["y"], runs[False][1]["y"])
    assert ey < 1e-5


def test_bf6_refine_layers_match_native():
    """MultiScaleRefine alone (bs 2, 256x256, eval) on one fixed input, bf16x6 against the native fp32 MFMA, layer by
    layer (every conv output with a fused PReLU, in forward order) and the traced stages, with the three scales on
    their branch streams and serialised; the path has no discontinuity."""
    from hyres_hip import ops as O
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    D = dev()
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(D).eval()
    x = torch.rand((2, 3, 256, 256), generator=torch.Generator().manual_seed(3)).to(D)
    runs = {}
    for on in (False, True):
        O.Trace.nodes, O.Trace.acts = {}, []
        with _Bf6(on), torch.no_grad():
            out = net.refine.hip(None, O.to_nhwc(x))
            res = O.to_nchw(out).double().cpu()
        torch.cuda.synchronize()
        runs[on] = ([(tuple(n.v.shape), O.to_nchw(n).double().cpu()) for _, n, _ in O.Trace.acts],
                    {k: O.Trace.value(k).double().cpu() for k in O.Trace.nodes}, res)
        O.Trace.nodes, O.Trace.acts = None, None
    a, b = runs[False][0], runs[True][0]
    rows = [(i, a[i][0], rel_err(b[i][1], a[i][1])) for i in range(len(a))]
    print("refine layers (index, NHWC shape, bf16x6 vs native):", [(i, s, f"{e:.1e}") for i, s, e in rows])
    for k in runs[False][1]:
        print(f"stage {k}: bf16x6 vs native {rel_err(runs[True][1][k], runs[False][1][k]):.2e}")
    e = rel_err(runs[True][2], runs[False][2])
    print(f"refine output: {e:.2e}")
    from hyres_hip import _lib as L
    g2 = O._geom("hyres_geom_conv2d", 2, 128, 128, 64, 64, 64, 64, 3, 3, 1, 1, 1)
    e2 = L.Epilogue()
    e2.kind, e2.act = L.EPI_BIAS, L.ACT_PRELU
    with _Bf6(True):
        print("1/2-scale first conv kernel under bf16x6:", O.conv_variant(g2, e2, O.conv_split(g2, e2) > 1))
    # bf16x6 with branches three more times: the 1/2-scale block's input (the bilinear output) and first conv
    reps = []
    for _ in range(3):
        O.Trace.nodes, O.Trace.acts = {}, []
        with _Bf6(True), torch.no_grad():
            net.refine.hip(None, O.to_nhwc(x))
        torch.cuda.synchronize()
        reps.append((O.Trace.value("refine_f2_in").double().cpu(), O.to_nchw(O.Trace.acts[3][1]).double().cpu()))
        O.Trace.nodes, O.Trace.acts = None, None
    print("bf6 branches, reps vs first: f2 input %s, layer 3 %s" % (
        ["%.1e" % rel_err(r[0], reps[0][0]) for r in reps[1:]], ["%.1e" % rel_err(r[1], reps[0][1]) for r in reps[1:]]))
    # the same with the three scales serialised on one stream, and bf16x6 twice (run-to-run)
    extra = {}
    for tag, on, branches in (("bf6_serial", True, False), ("native_serial", False, False), ("bf6_again", True, True)):
        O.BranchStreams.enabled = branches
        try:
            with _Bf6(on), torch.no_grad():
                extra[tag] = O.to_nchw(net.refine.hip(None, O.to_nhwc(x))).double().cpu()
            torch.cuda.synchronize()
        finally:
            O.BranchStreams.enabled = True
    print("bf6 serial vs native serial %.2e, bf6 serial vs native branches %.2e, bf6 branches run-to-run %.2e, "
          "native serial vs native branches %.2e" % (rel_err(extra["bf6_serial"], extra["native_serial"]),
                                                     rel_err(extra["bf6_serial"], runs[False][2]),
                                                     rel_err(extra["bf6_again"], runs[True][2]),
                                                     rel_err(extra["native_serial"], runs[False][2])))
    # bf16x6 agrees with native to fp32 noise serialised and with the branch streams, and each is the same run to run
    # (round 4 found the bf16x6 weight-resident conv corrupting co-resident waves of the branch kernels: 4e-2 here)
    assert rel_err(runs[True][2], runs[False][2]) < 1e-5
    assert rel_err(extra["bf6_again"], runs[True][2]) == 0.0
    assert all(rel_err(r[0], reps[0][0]) == 0.0 and rel_err(r[1], reps[0][1]) == 0.0 for r in reps[1:])
    assert rel_err(extra["bf6_serial"], extra["native_serial"]) < 1e-5
    assert rel_err(extra["native_serial"], runs[False][2]) < 1e-6


@pytest.mark.parametrize("case", [
    # (B, H, W, Ci, Co, k, out channels of the host buffer, channel offset) — the MultiScaleRefine / latent convs
    (2, 256, 256, 64, 64, 3, 192, 0), (2, 256, 256, 64, 64, 3, 64, 0), (2, 128, 128, 64, 64, 3, 192, 64),
    (2, 64, 64, 64, 64, 3, 192, 128), (2, 128, 128, 64, 64, 3, 64, 0), (1, 64, 96, 384, 640, 1, 640, 0),
    (1, 64, 96, 640, 512, 1, 512, 0)])
def test_bf6_writes_stay_inside_the_output(case):
    """Every bf16x6 conv writes its output view and nothing else: the view sits inside a sentinel-filled buffer (one
    image before and after it, the other channels of a wider pixel stride), which must be untouched after the conv."""
    from hyres_hip import ops as O
    D = dev()
    B, H, W, Ci, Co, k, Cb, c0 = case
    x = O.to_nhwc(_rand((B, Ci, H, W), 61).to(D))
    w = torch.nn.Parameter(_rand((Co, Ci, k, k), 62, (Ci * k * k) ** -0.5).to(D))
    b = _rand((Co,), 63, 0.1).to(D)
    slope = torch.full((1,), 0.25, device=D)
    for on in (False, True):
        big = torch.full((B + 2, H, W, Cb), 12345.0, device=D)
        out = O.Node(big[1:B + 1, ..., c0:c0 + Co])
        with _Bf6(on), torch.no_grad():
            O.conv2d(None, x, w, b, pad=k // 2, act=L_ACT_PRELU(), slope=slope, out=out)
        torch.cuda.synchronize()
        keep = torch.ones_like(big, dtype=torch.bool)
        keep[1:B + 1, ..., c0:c0 + Co] = False
        bad = int((big[keep] != 12345.0).sum())
        print(case, "bf16x6" if on else "native", "writes outside the view:", bad)
        assert bad == 0


def L_ACT_PRELU():
    from hyres_hip import _lib as L
    return L.ACT_PRELU


def test_bf6_refine_branch_determinism():
    """MultiScaleRefine (bs 2, 256x256, eval) with its branch streams, bf16x6 switched on for a subset of the three
    scales (the others native), three runs each: the run-to-run spread of the 1/2-scale input and of the output."""
    from hyres_hip import ops as O
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    D = dev()
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(D).eval()
    x = torch.rand((2, 3, 256, 256), generator=torch.Generator().manual_seed(3)).to(D)
    rf = net.refine
    seqs = [rf.scale1, rf.scale2, rf.scale3]
    origs = [s.hip for s in seqs]

    def wrap(fn, on):
        def hip(*a, **kw):
            with _Bf6(on):
                return fn(*a, **kw)
        return hip
    rows = []
    try:
        for subset in ((), (0,), (1,), (2,), (1, 2), (0, 1, 2)):
            for i, s in enumerate(seqs):
                s.hip = wrap(origs[i], i in subset)
            reps = []
            for _ in range(3):
                O.Trace.nodes, O.Trace.acts = {}, []
                with torch.no_grad():
                    out = rf.hip(None, O.to_nhwc(x))
                torch.cuda.synchronize()
                reps.append((O.Trace.value("refine_f2_in").double().cpu(), O.to_nchw(out).double().cpu()))
                O.Trace.nodes, O.Trace.acts = None, None
            rows.append((subset, max(rel_err(r[0], reps[0][0]) for r in reps[1:]),
                         max(rel_err(r[1], reps[0][1]) for r in reps[1:])))
    finally:
        for i, s in enumerate(seqs):
            s.hip = origs[i]
    for subset, ef, eo in rows:
        print(f"bf16x6 on scales {[i + 1 for i in subset]}: run-to-run f2 input {ef:.1e}, output {eo:.1e}")
    assert all(ef == 0.0 and eo == 0.0 for _, ef, eo in rows)


@pytest.mark.parametrize("mode", ["native", "bf16x6", "f16"])
def test_conv_beside_side_stream_kernels(mode):
    """Which side-stream results change while a full-scale 3x3 conv (conv3x3_wres_*) runs on the main stream: a
    bilinear of the conv's own input, a bilinear of an unrelated tensor, a plain copy of an unrelated tensor; and the
    conv's own output. Each against the same kernel run alone."""
    from hyres_hip import ops as O
    from hyres_hip import refine_ops as R
    D = dev()
    B, H, W, C = 2, 256, 256, 64
    half = mode == "f16"
    dt = torch.float16 if half else torch.float32
    feat = O.Node(O.to_nhwc(_rand((B, C, H, W), 71).to(D)).v.to(dt).contiguous())
    other = O.Node(O.to_nhwc(_rand((B, C, H, W), 74).to(D)).v.to(dt).contiguous())
    w = torch.nn.Parameter(_rand((C, C, 3, 3), 72, (C * 9) ** -0.5).to(D))
    b = _rand((C,), 73, 0.1).to(D)
    slope = torch.full((1,), 0.25, device=D)
    side = torch.cuda.Stream(device=D)

    def conv():
        with torch.autocast("cuda", dtype=torch.float16, enabled=half):
            return O.conv2d(None, feat, w, b, pad=1, act=L_ACT_PRELU(), slope=slope)

    def sides():
        return (R.bilinear(None, feat, H // 2, W // 2, 2.0, 2.0).v, R.bilinear(None, other, H // 2, W // 2, 2.0, 2.0).v,
                other.v.clone())
    with _Bf6(mode == "bf16x6"), torch.no_grad():
        y0 = conv().v.clone()
        ref = [t.clone() for t in sides()]
        torch.cuda.synchronize()
        worst = [0.0] * 4
        for _ in range(5):
            fork = torch.cuda.Event()
            fork.record()
            y = conv()
            side.wait_event(fork)
            with torch.cuda.stream(side):
                got = sides()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            for i, (g_, r_) in enumerate(zip(got, ref)):
                worst[i] = max(worst[i], (g_.float() - r_.float()).abs().max().item())
            worst[3] = max(worst[3], (y.v.float() - y0.float()).abs().max().item())
    print(f"{mode}: max |diff| vs alone — bilinear(conv input) {worst[0]:.2e}, bilinear(other) {worst[1]:.2e}, "
          f"copy(other) {worst[2]:.2e}, conv output {worst[3]:.2e}")
    assert worst == [0.0] * 4


def test_bf6_kernels_beside_a_bilinear():
    """Each bf16x6 kernel family (and its native counterpart) on the main stream while a side stream resamples an
    unrelated tensor three times: the largest change of the resampled values against the same resampling alone."""
    from hyres_hip import ops as O
    from hyres_hip import refine_ops as R
    D = dev()
    other = O.to_nhwc(_rand((2, 64, 256, 256), 74).to(D))
    side = torch.cuda.Stream(device=D)
    slope = torch.full((1,), 0.25, device=D)
    with torch.no_grad():
        ref = R.bilinear(None, other, 128, 128, 2.0, 2.0).v.clone()
    torch.cuda.synchronize()

    def fwd(B, H, W, Ci, Co, k, dil=1, bwd=False):
        x = O.to_nhwc(_rand((B, Ci, H, W), 75).to(D), rg=bwd)
        w = torch.nn.Parameter(_rand((Co, Ci, k, k), 76, (Ci * k * k) ** -0.5).to(D))
        b = torch.nn.Parameter(_rand((Co,), 77, 0.1).to(D))
        gy = O.nchw_grad_to_nhwc(_rand((B, Co, H, W), 78).to(D)) if bwd else None

        def run():
            tape = O.Tape() if bwd else None
            y = O.conv2d(tape, x, w, b, pad=dil * (k // 2), dil=dil, act=L_ACT_PRELU(), slope=slope)
            if bwd:
                y.set_grad(gy)
                tape.backward()
        return run
    cases = {"3x3 2x256² (weight-resident)": fwd(2, 256, 256, 64, 64, 3),
             "3x3 dil2 2x256² (implicit GEMM)": fwd(2, 256, 256, 64, 64, 3, 2),
             "3x3 2x128² (implicit GEMM)": fwd(2, 128, 128, 64, 64, 3),
             "1x1 64x96 384->640": fwd(1, 64, 96, 384, 640, 1),
             "3x3 2x128² fwd+bwd (dgrad, halo wgrad)": fwd(2, 128, 128, 64, 64, 3, bwd=True),
             "1x1 2x128² 128->64 fwd+bwd (1x1 wgrad)": fwd(2, 128, 128, 128, 64, 1, bwd=True)}
    for name, run in cases.items():
        for on in (False, True):
            worst = 0.0
            with _Bf6(on):
                run()
                torch.cuda.synchronize()
                for _ in range(4):
                    fork = torch.cuda.Event()
                    fork.record()
                    with torch.no_grad() if "bwd" not in name else torch.enable_grad():
                        run()
                    side.wait_event(fork)
                    with torch.cuda.stream(side), torch.no_grad():
                        got = [R.bilinear(None, other, 128, 128, 2.0, 2.0).v for _ in range(3)]
                    torch.cuda.current_stream().wait_stream(side)
                    torch.cuda.synchronize()
                    worst = max([worst] + [(g_ - ref).abs().max().item() for g_ in got])
            print(f"{name:42s} {'bf16x6' if on else 'native'}: side-stream bilinear max |diff| vs alone {worst:.2e}")
            assert worst == 0.0, (name, on)


@pytest.mark.parametrize("variant", [1, 2, 3])
def test_wres_bf6_variants_bit_identical(variant):
    """conv3x3_wres_bf6_kernel's scheduling variants (hyres_conv_tuning key 12: bit 0 the hand-pipelined fragment
    reads, bit 1 static priority for waves 4..7) change only WHEN the LDS reads issue, not the MFMA order: the output
    must equal variant 0 bit for bit (128^2 with residual + ReLU, and a Kodak-size image with PReLU)."""
    import ctypes
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    C = 64
    slope = torch.tensor([0.25], device=D)
    for (B, H, W, act) in [(4, 128, 128, "relu"), (1, 512, 768, "prelu")]:
        x = _rand((B, C, H, W), 51).to(D)
        w = torch.nn.Parameter(_rand((C, C, 3, 3), 52, (C * 9) ** -0.5).to(D))
        b = _rand((C,), 53, 0.1).to(D)
        r = _rand((B, C, H, W), 54).to(D)
        a = L.ACT_RELU if act == "relu" else L.ACT_PRELU
        outs = {}
        for v in (0, variant):
            old = ctypes.c_int(0)
            with _Bf6(True):
                L.call("hyres_conv_tuning", 12, v, ctypes.byref(old))
                try:
                    xn, rn = O.to_nhwc(x), O.to_nhwc(r)
                    yn = O.conv2d(None, xn, w, b, pad=1, act=a, res=rn, slope=slope if act == "prelu" else None)
                    outs[v] = O.to_nchw(yn).clone()
                finally:
                    L.call("hyres_conv_tuning", 12, old.value, None)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[variant]), (B, H, W, act, (outs[0] - outs[variant]).abs().max().item())



@pytest.mark.parametrize("autocast", [False, True])
def test_refine_sa_mul_fold_matches_unfused(autocast):
    """Inference MultiScaleRefine with SpatialAttention's multiply folded into fusion[0]'s epilogue
    (models/layers/enhancement.py FOLD_SA_MUL, HYRES_EPI_ROWSCALE: attn[p] * conv_nobias(multi) + bias) against the
    unfused multiply-then-conv, on the full model's refine output at 2 x 64 x 96 (fp32: 1e-6 normwise, the
    reassociation of one fp32 multiply; autocast with fp16 activations: 2e-3, the fp16 rounding of multi * attn the
    unfused path stores)."""
    import models.layers.enhancement as EH
    from hyres_hip import ops as O
    from models import ResidualJPEGCompression
    from hyres_hip.weights import synthetic_state_dict
    D = dev()
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(D).eval()
    g = torch.Generator().manual_seed(7)
    x = (torch.randint(0, 256, (2, 3, 64, 96), generator=g).float() / 255)
    jpeg, bpp = net.jpeg(x)
    outs = {}
    for fold in (False, True):
        EH.FOLD_SA_MUL = fold
        try:
            ctx = torch.autocast("cuda", dtype=torch.float16) if autocast else torch.autocast("cuda", enabled=False)
            with torch.no_grad(), ctx:
                outs[fold] = net.forward_device(x.to(D), jpeg.to(D), bpp)["x_hat"].double().cpu()
        finally:
            EH.FOLD_SA_MUL = True
    err = rel_err(outs[True], outs[False])
    print("autocast" if autocast else "fp32", f"x_hat folded vs unfused: {err:.2e}")
    assert err < (2e-3 if autocast else 1e-6)


@pytest.mark.parametrize("kind,B,Ci,H,W,f16x", [
    ("conv3x3", 3, 64, 67, 132, False),    # MultiScaleRefine.fusion[2] (64 -> 3), partial last block
    ("conv3x3", 2, 128, 45, 76, False),
    ("deconv5x5", 2, 128, 33, 48, False),  # g_s's last deconv (128 -> 3: four phases, descending tap grids)
    ("conv3x3", 2, 64, 40, 72, True),      # fp16 activations (autocast inference)
    ("deconv5x5", 2, 128, 20, 36, True),
])
def test_narrow_strip_kernel_matches_fp64(kind, B, Ci, H, W, f16x):
    """conv_narrow_strip_kernel (Co <= 4, 4-pixel strips with the inputs loaded once per strip and the weights in
    VGPRs, hyres_conv_tuning key 13 = 1) against float64 torch and no worse than twice conv_narrow_kernel (key 13 = 0),
    for MultiScaleRefine's 3x3 64 -> 3 and g_s's 5x5 stride-2 deconv 128 -> 3, fp32 and fp16 inputs, Co in {3, 1},
    plus the accumulate epilogue (y += conv) the input-gradient path uses."""
    import ctypes
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    for Co in (3, 1):
        x = _rand((B, Ci, H, W), 81).to(D)
        if f16x:
            x = x.half().float()
        if kind == "conv3x3":
            w = _rand((Co, Ci, 3, 3), 82, (Ci * 9) ** -0.5).to(D)
            b = _rand((Co,), 83, 0.1).to(D)
            ref = F.conv2d(x.double(), w.double(), b.double(), padding=1)
        else:
            w = _rand((Ci, Co, 5, 5), 82, (Ci * 25 / 4) ** -0.5).to(D)
            b = _rand((Co,), 83, 0.1).to(D)
            ref = F.conv_transpose2d(x.double(), w.double(), b.double(), stride=2, padding=2, output_padding=1)
        errs, names = {}, {}
        for key in (1, 0):
            old = ctypes.c_int(0)
            L.call("hyres_conv_tuning", 13, key, ctypes.byref(old))
            try:
                xn = O.to_nhwc(x)
                if f16x:
                    xn = O.Node(xn.v.half(), rg=False)
                if kind == "conv3x3":
                    yn = O.conv2d(None, xn, torch.nn.Parameter(w), b, pad=1)
                    g = O._geom("hyres_geom_conv2d", B, H, W, Ci, Ci, Co, Co, 3, 3, 1, 1, 1)
                else:
                    yn = O.deconv2d(None, xn, torch.nn.Parameter(w), b)
                    g = O._geom("hyres_geom_deconv2d", B, H, W, Ci, Ci, Co, Co, 5, 2, 1)
                e = L.Epilogue()
                e.io_f16 = L.IO_X16 if f16x else 0
                names[key] = O.conv_variant(g, e, False)
                y = O.to_nchw(yn).double()
                torch.cuda.synchronize()
            finally:
                L.call("hyres_conv_tuning", 13, old.value, None)
            errs[key] = rel_err(y.cpu(), ref.cpu())
        print(kind, B, Ci, H, W, f16x, Co, names, f"error vs fp64: strip {errs[1]:.2e}, per-pixel {errs[0]:.2e}")
        assert names[1].startswith("conv_narrow_strip_kernel") and names[0].startswith("conv_narrow_kernel"), names
        assert errs[1] < 1e-5 and errs[1] <= 2 * errs[0] + 1e-9


@pytest.mark.parametrize("B,H,W,act", [(4, 128, 128, "relu"), (1, 256, 384, "prelu"), (1, 256, 384, "relu"),
                                       (4, 128, 128, "prelu"), (2, 128, 256, "prelu")])
def test_wres_bf6_dilation2_matches_fp64(B, H, W, act):
    """The weight-resident bf16x6 3x3 at halo radius 2 (conv3x3_wres_bf6_kernel<true, 1, 2>: MultiScaleRefine's
    dilation-2 convs, enhancement.py:44-51) — forward with residual and the input gradient (a dilation-2 conv over dY)
    — against float64 torch, and no worse than twice the implicit GEMM it replaces (hyres_conv_tuning key 14 = 0)."""
    import ctypes
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    C = 64
    x = _rand((B, C, H, W), 91)
    w = _rand((C, C, 3, 3), 92, (C * 9) ** -0.5)
    b = _rand((C,), 93, 0.1)
    r = _rand((B, C, H, W), 94)
    gy = _rand((B, C, H, W), 95)
    xr = x.double().requires_grad_()
    pre = F.conv2d(xr, w.double(), b.double(), padding=2, dilation=2) + r.double()
    yr = F.relu(pre) if act == "relu" else torch.where(pre >= 0, pre, 0.25 * pre)
    yr.backward(gy.double())
    slope = torch.tensor([0.25], device=D)
    a = L.ACT_RELU if act == "relu" else L.ACT_PRELU
    res, names = {}, {}
    for key in (1, 0):
        old = ctypes.c_int(0)
        L.call("hyres_conv_tuning", 14, key, ctypes.byref(old))
        try:
            tape = O.Tape()
            xn = O.to_nhwc(x.to(D), rg=True)
            rn = O.to_nhwc(r.to(D))
            wd = torch.nn.Parameter(w.to(D))
            yn = O.conv2d(tape, xn, wd, b.to(D), pad=2, dil=2, act=a, slope=slope if act == "prelu" else None, res=rn)
            yn.set_grad(O.nchw_grad_to_nhwc(gy.to(D)))
            tape.backward()
            torch.cuda.synchronize()
            g = O._geom("hyres_geom_conv2d", B, H, W, C, C, C, C, 3, 3, 1, 2, 2)
            e = L.Epilogue()
            e.kind, e.act = L.EPI_BIAS, a
            names[key] = O.conv_variant(g, e, False)
            res[key] = (O.to_nchw(yn).double().cpu(), O.to_nchw_grad(xn).double().cpu())
        finally:
            L.call("hyres_conv_tuning", 14, old.value, None)
    ey = {k: rel_err(v[0], yr.detach()) for k, v in res.items()}
    # dx against the float64 conv input-gradient of dY masked by OUR activation: at 6.3M outputs a few land within
    # fp32 rounding of 0, where a float64-masked reference flips whole gradient entries (seen: 2.5e-2 for both kernels)
    def dx_ref(y):
        gp = gy.double() * torch.where(y > 0, 1.0, 0.0 if act == "relu" else 0.25)
        return torch.nn.grad.conv2d_input(x.shape, w.double(), gp, padding=2, dilation=2)
    eg = {k: rel_err(v[1], dx_ref(v[0])) for k, v in res.items()}
    print("dx vs float64-masked reference:", {k: f"{rel_err(v[1], xr.grad):.2e}" for k, v in res.items()})
    print(B, H, W, act, names, f"y vs fp64: wres {ey[1]:.2e}, igemm {ey[0]:.2e}; dx: wres {eg[1]:.2e}, igemm {eg[0]:.2e}")
    assert names[1] == "conv3x3_wres_bf6_kernel" and names[0] != names[1], names
    assert ey[1] < 1e-5 and ey[1] <= 2 * ey[0] + 1e-9
    assert eg[1] < 1e-5 and eg[1] <= 2 * eg[0] + 1e-9


@pytest.mark.parametrize("K,B,H,W,Ci,Co,key,S", [
    (1, 2, 30, 30, 96, 160, 15, 1),    # 1x1: ragged pixel chunks (1800 px) and channel tiles
    (1, 4, 64, 64, 64, 128, 15, 1),
    (1, 2, 128, 128, 128, 64, 15, 1),
    (3, 2, 64, 64, 64, 64, 16, 1),     # 3x3 rows of taps on the halo kernel
    (3, 3, 32, 96, 96, 96, 16, 1),     # 96 channels: a partial 64-wide tile
    (3, 2, 128, 128, 64, 128, 16, 1),
    (5, 2, 64, 64, 128, 128, 16, 2),   # round 6: 5-tap rows, stride 2 (g_a / h_a's 5x5 s2 convs)
    (5, 2, 32, 32, 96, 96, 16, 1),     # 5-tap rows, stride 1 (the masked 5x5 context conv's shape)
])
def test_wgrad_prefetch2_kernels_bit_identical(K, B, H, W, Ci, Co, key, S):
    """wgrad1x1_bf6_pf2_kernel (hyres_conv_tuning key 15) and wgrad_halo_bf6_pf2_kernel (key 16): operand loads two
    32-pixel chunks ahead through unconditional buffer loads — the same products in the same order as the one-ahead
    kernels, so weight and bias gradients are equal bit for bit (ragged chunks and tiles included), and within fp32
    accuracy of the fp64 reference (reference: the weight gradients of models/layers/attention.py:11-30's convs)."""
    import ctypes
    from hyres_hip import _lib as L
    D = dev()
    g = torch.Generator().manual_seed(5)
    x = (torch.rand((B, H, W, Ci), generator=g) * 2 - 1).to(D)
    gy = (torch.rand((B, H // S, W // S, Co), generator=g) * 2 - 1).to(D)
    d = L.WgradDesc()
    L.call("hyres_wgrad_desc_conv2d", ctypes.byref(d), B, H, W, Ci, Ci, Co, Co, K, K, S, K // 2, 1)
    d.sm = Ci * K * K
    nb = L.load().hyres_wgrad_workspace_bytes(ctypes.byref(d))
    ws = torch.empty(nb // 4 + 16, device=D)
    old = ctypes.c_int(0)
    L.call("hyres_conv_tuning", 7, 1, ctypes.byref(old))
    res = {}
    try:
        for v in (1, 2):
            L.call("hyres_conv_tuning", key, v, None)
            dw = torch.zeros((Co, Ci, K, K), device=D)
            db = torch.zeros((Co,), device=D)
            L.call("hyres_conv_wgrad", ctypes.byref(d), gy.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(),
                   ws.data_ptr(), nb, L.stream())
            torch.cuda.synchronize()
            res[v] = (dw.cpu(), db.cpu())
    finally:
        L.call("hyres_conv_tuning", key, 2, None)
        L.call("hyres_conv_tuning", 7, old.value, None)
    assert torch.equal(res[1][0], res[2][0]) and torch.equal(res[1][1], res[2][1])
    xr = x.cpu().double().permute(0, 3, 1, 2)
    gr = gy.cpu().double().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xr, (Co, Ci, K, K), gr, stride=S, padding=K // 2)
    err = float((res[2][0].double() - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err
    assert float((res[2][1].double() - gr.sum((0, 2, 3))).abs().max()) < 1e-3


@pytest.mark.parametrize("B,H,Ci,Co,K,stride,swz_off", [
    (16, 32, 96, 96, 3, 1, False),     # AttentionBlock(192)'s RU 3x3 at 32^2 (the 64x64 tile)
    (16, 32, 192, 96, 1, 1, False),    # its 1x1 192 -> 96
    (4, 64, 128, 128, 5, 2, False),    # 5x5 stride 2 (g_a)
    (2, 16, 384, 192, 3, 1, True),     # a split-K grid; and the 80-B padded rows (key 19 = 0) as the reference
])
def test_bf6_implicit_gemm_staging_variants_bit_identical(B, H, Ci, Co, K, stride, swz_off):
    """The bf16x6 implicit GEMM's LDS staging variants change where the split planes sit and when they are stored,
    not the MFMAs or their order: the double-buffered 64x64-tile kernel (hyres_conv_tuning key 20 = 1,
    conv_fwd_b6db_kernel) and the XOR-swizzled 64-B rows (key 19, default) must equal the single-buffered kernel and
    (swz_off) the 80-B padded rows bit for bit — forward with bias + ReLU and the residual epilogue."""
    import ctypes
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    x = _rand((B, Ci, H, H), 71).to(D)
    w = torch.nn.Parameter(_rand((Co, Ci, K, K), 72, (Ci * K * K) ** -0.5).to(D))
    b = _rand((Co,), 73, 0.1).to(D)
    Ho = H // stride
    r = _rand((B, Co, Ho, Ho), 74).to(D)

    def run(db, sw):
        olds = [ctypes.c_int(0), ctypes.c_int(0)]
        with _Bf6(True):
            L.call("hyres_conv_tuning", 20, db, ctypes.byref(olds[0]))
            L.call("hyres_conv_tuning", 19, sw, ctypes.byref(olds[1]))
            try:
                xn, rn = O.to_nhwc(x), O.to_nhwc(r)
                yn = O.conv2d(None, xn, w, b, stride=stride, pad=K // 2, act=L.ACT_RELU, res=rn)
                torch.cuda.synchronize()
                return O.to_nchw(yn).clone()
            finally:
                L.call("hyres_conv_tuning", 20, olds[0].value, None)
                L.call("hyres_conv_tuning", 19, olds[1].value, None)

    ref = run(0, 0 if swz_off else 1)
    for db, sw in ((1, 1), (0, 1)):
        got = run(db, sw)
        assert torch.equal(ref, got), (db, sw, float((ref - got).abs().max()))


@pytest.mark.parametrize("B,H,W,Ci,Co", [(2, 64, 96, 3, 64), (2, 48, 256, 64, 3), (1, 37, 200, 3, 64)])
def test_wgrad_thin_window_bit_identical(B, H, W, Ci, Co):
    """wgrad_thin_kernel's sliding 3x3 Q window (round 6, hyres_conv_tuning key 23): the same FMAs per accumulator in
    the same pixel order as the nine-reads-per-pixel loop, so the weight and bias gradients of the image-side 3x3 convs
    (MultiScaleRefine's conv_in 3 -> 64 and its output conv 64 -> 3, through the swapped descriptor) are equal bit for
    bit, on ragged widths (a partial last 64-pixel chunk), and within 1e-5 of fp64."""
    import ctypes
    from hyres_hip import _lib as L
    D = dev()
    g = torch.Generator().manual_seed(9)
    x = (torch.rand((B, H, W, Ci), generator=g) * 2 - 1).to(D)
    gy = (torch.rand((B, H, W, Co), generator=g) * 2 - 1).to(D)
    d = L.WgradDesc()
    L.call("hyres_wgrad_desc_conv2d", ctypes.byref(d), B, H, W, Ci, Ci, Co, Co, 3, 3, 1, 1, 1)
    d.sm = Ci * 9
    nb = L.load().hyres_wgrad_workspace_bytes(ctypes.byref(d))
    ws = torch.empty(nb // 4 + 16, device=D)
    res = {}
    try:
        for v in (0, 1):
            L.call("hyres_conv_tuning", 23, v, None)
            dw = torch.zeros((Co, Ci, 3, 3), device=D)
            db = torch.zeros((Co,), device=D)
            L.call("hyres_conv_wgrad", ctypes.byref(d), gy.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(),
                   ws.data_ptr(), nb, L.stream())
            torch.cuda.synchronize()
            res[v] = (dw.cpu(), db.cpu())
    finally:
        L.call("hyres_conv_tuning", 23, 1, None)
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    ref = torch.nn.grad.conv2d_weight(x.cpu().double().permute(0, 3, 1, 2), (Co, Ci, 3, 3),
                                      gy.cpu().double().permute(0, 3, 1, 2), padding=1)
    assert float((res[1][0].double() - ref).abs().max() / ref.abs().max()) < 1e-5
