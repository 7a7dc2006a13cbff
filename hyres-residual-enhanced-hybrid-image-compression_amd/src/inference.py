"""Inference CLI (src/inference.py:18-253) — same flags; HIP forward path, rANS compress/decompress.

Per image (as the reference, :53-150): ``model.compress(x)`` -> ``model.decompress(...)``; y/z bpp from
the rANS string lengths, JPEG bpp from the real JPEG bytes, enc/dec time from the models' own timers.
PSNR = 10*log10(1/mse) — the reference's formula at :123-125, ``-10*log10(mse*255^2)``, is wrong (it
would report a large negative number); fixed here and documented in DESIGN.md.
CSV columns are the reference's (:232-246)."""
import argparse
import csv
import math
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
from PIL import Image

from models import LightWeightCheckerboard, ResidualJPEGCompression
from src.utils import load_checkpoint


def parse_args(argv):
    p = argparse.ArgumentParser(description="Inference script for ResidualJPEGCompression model.")
    p.add_argument("--checkpoint", type=str, required=True, help="Path to the checkpoint model")
    p.add_argument("--input", type=str, required=True, help="Path to input image or directory of images")
    p.add_argument("--output", type=str, default="./output", help="Output directory path")
    p.add_argument("--N", type=int, default=128, help="Number of channels (default: %(default)s)")
    p.add_argument("--M", type=int, default=192, help="Number of latent channels (default: %(default)s)")
    p.add_argument("--jpeg-quality", default=1, type=int, help="JPEG quality factor (default: %(default)s)")
    p.add_argument("--cuda", type=lambda x: str(x).lower() == "true", default=True,
                   help="Use cuda if available (default: %(default)s)")
    p.add_argument("--save-components", action="store_true", help="Save JPEG and residual components")
    return p.parse_args(argv)


def _load_image(path):
    a = np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8)
    return torch.from_numpy(a.copy()).permute(2, 0, 1).float().div(255.0).unsqueeze(0)


def _save(t, path):
    a = (t[0].detach().clamp(0, 1).permute(1, 2, 0).cpu().numpy() * 255 + 0.5).astype(np.uint8)
    Image.fromarray(a).save(path)


def process_image(model, img_path, output_dir, device, save_components=False):
    """src/inference.py:53-150: compress -> decompress, bpp from the real strings (rANS + JPEG bytes)."""
    x = _load_image(img_path)
    H, W = x.shape[-2:]
    if H % 32 or W % 32:
        raise ValueError(f"{img_path}: H and W must be multiples of 32 (g_a /8 then h_a /4)")
    num_pixels = x.size(0) * H * W
    x = x.to(device)
    out_enc = model.compress(x)
    torch.cuda.synchronize()
    enc_time = out_enc["time"]
    out_dec = model.decompress(out_enc)
    torch.cuda.synchronize()
    dec_time = out_dec["time"]
    base, ext = os.path.splitext(os.path.basename(img_path))
    _save(out_dec["x_hat"], os.path.join(output_dir, f"{base}_recon{ext}"))
    with torch.no_grad():
        out_net = model(x)
    if save_components:
        _save(x, os.path.join(output_dir, f"{base}_original{ext}"))
        _save(out_net["jpeg_decoded"], os.path.join(output_dir, f"{base}_jpeg{ext}"))
        _save(out_net["residual"] * 0.5 + 0.5, os.path.join(output_dir, f"{base}_residual{ext}"))
        _save(out_net["residual_hat"] * 0.5 + 0.5, os.path.join(output_dir, f"{base}_residual_hat{ext}"))
    y_bpp = sum(len(s) * 8 for part in out_enc["strings"][0] for s in part) / num_pixels
    z_bpp = sum(len(s) * 8 for s in out_enc["strings"][1]) / num_pixels
    jpeg_bpp = float(out_net["jpeg_bpp_loss"])
    total_bpp = jpeg_bpp + y_bpp + z_bpp
    mse = torch.nn.functional.mse_loss(x, out_dec["x_hat"]).item()
    psnr = 10 * math.log10(1.0 / max(mse, 1e-12))
    print(f"Processed {img_path}")
    print(f"Total bpp: {total_bpp:.4f} (JPEG: {jpeg_bpp:.4f}, Y: {y_bpp:.5f}, Z: {z_bpp:.5f})")
    print(f"MSE: {mse * 255 ** 2:.4f})")
    print(f"PSNR: {psnr:.2f} dB, MS-SSIM: 0.0000")
    print(f"Encoding time: {enc_time:.4f}s, Decoding time: {dec_time:.4f}s")
    return {"filename": os.path.basename(img_path), "total_bpp": total_bpp, "jpeg_bpp": jpeg_bpp, "y_bpp": y_bpp,
            "z_bpp": z_bpp, "mse": mse * 255 ** 2, "psnr": psnr, "ms_ssim": 0.0, "enc_time": enc_time,
            "dec_time": dec_time}


def main(argv):
    args = parse_args(argv)
    if not torch.cuda.is_available():
        raise RuntimeError("the HIP path needs a ROCm GPU")
    device = torch.device("cuda")
    os.makedirs(args.output, exist_ok=True)
    ckpt = Path(args.checkpoint).resolve()
    if not ckpt.is_file():
        raise RuntimeError(f'"{ckpt}" is not a valid file.')
    state_dict = load_checkpoint(ckpt)
    model = ResidualJPEGCompression(base_model=LightWeightCheckerboard(N=args.N, M=args.M),
                                    jpeg_quality=args.jpeg_quality)
    model.load_state_dict(state_dict)
    model = model.to(device).eval()
    model.update()  # CDF tables (no-op for a checkpoint saved after update(), src/updata.py)
    inp = Path(args.input).resolve()
    if inp.is_file():
        paths = [inp]
    elif inp.is_dir():
        paths = sorted(p for p in inp.glob("*") if p.suffix.lower() in (".jpg", ".jpeg", ".png", ".bmp"))
    else:
        raise RuntimeError(f'"{inp}" is neither a file nor a directory.')
    metrics = [process_image(model, str(p), args.output, device, args.save_components) for p in paths]
    if metrics:
        keys = [k for k in metrics[0] if k != "filename"]
        avg = {k: sum(m[k] for m in metrics) / len(metrics) for k in keys}
        print("\nAverage metrics:")
        print(f"Total bpp: {avg['total_bpp']:.4f} (JPEG: {avg['jpeg_bpp']:.4f}, Y: {avg['y_bpp']:.5f}, "
              f"Z: {avg['z_bpp']:.5f})")
        print(f"PSNR: {avg['psnr']:.2f} dB")
        with open(os.path.join(args.output, "metrics.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["filename", "total_bpp", "jpeg_bpp", "y_bpp", "z_bpp", "mse", "psnr", "ms_ssim",
                        "enc_time(s)", "dec_time(s)"])
            for m in metrics:
                w.writerow([m["filename"], m["total_bpp"], m["jpeg_bpp"], m["y_bpp"], m["z_bpp"], m["mse"],
                            m["psnr"], m["ms_ssim"], m["enc_time"], m["dec_time"]])


if __name__ == "__main__":
    main(sys.argv[1:])
