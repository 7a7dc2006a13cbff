"""Debug: one 1x1 conv with a ReLU-mask epilogue through the C-ABI vs torch, at a given pixel count."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd")]
import torch


def run(B, H, W, Ci, Co, act_mask, res, acc):
    from hyres_hip import _lib as L
    from hyres_hip.ops import _geom
    D = torch.device("cuda:0")
    torch.manual_seed(0)
    x = torch.randn(B, H, W, Ci, device=D)
    w = torch.randn(Co, Ci, device=D) / Ci ** 0.5
    m = torch.randn(B, H, W, Co, device=D).relu()
    r = torch.randn(B, H, W, Co, device=D)
    y0 = torch.randn(B, H, W, Co, device=D)
    y = y0.clone()
    g = _geom("hyres_geom_conv2d", B, H, W, Ci, Ci, Co, Co, 1, 1, 1, 0, 1)
    e = L.Epilogue()
    e.kind = L.EPI_BIAS
    ref = x.reshape(-1, Ci).double() @ w.double().t()
    if res:
        e.res = r.data_ptr(); e.ldres = Co
        ref = ref + r.reshape(-1, Co).double()
    if act_mask:
        e.act = L.ACT_RELU_MASK; e.aux0 = m.data_ptr(); e.ld0 = Co
        ref = torch.where(m.reshape(-1, Co) > 0, ref, torch.zeros_like(ref))
    if acc:
        e.accumulate = 1
        ref = ref + y0.reshape(-1, Co).double()
    nb = L.load().hyres_conv_workspace_bytes(ctypes.byref(g))
    ws = torch.empty(max(nb, 4) // 4 + 4, device=D)
    L.call("hyres_conv_forward", ctypes.byref(g), x.data_ptr(), w.data_ptr(), Ci, y.data_ptr(), ctypes.byref(e),
           ws.data_ptr(), nb, L.stream())
    torch.cuda.synchronize()
    err = (y.reshape(-1, Co).double() - ref).abs()
    bad = (err > 1e-4 * ref.abs().max()).nonzero()
    print(B, H, W, Ci, Co, "mask" if act_mask else "", "res" if res else "", "acc" if acc else "",
          "max err", float(err.max() / ref.abs().max()), "bad", bad.shape[0],
          "first bad rows", sorted(set(bad[:, 0].tolist()))[:8], "cols", sorted(set(bad[:, 1].tolist()))[:8])


if __name__ == "__main__":
    for shp in ((1, 183, 183, 64, 128), (1, 182, 182, 64, 128), (2, 183, 183, 128, 64)):
        for flags in ((1, 0, 0), (0, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0)):
            run(*shp, *flags)
