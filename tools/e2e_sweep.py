"""End-to-end Unrolled_ADMM (PyTorch ResUNet denoiser + HIP spectral engine) throughput sweep:
batch size x MIOpen find mode (torch.backends.cudnn.benchmark) x memory format.  One JSON line per
configuration, with the denoiser's share of the forward.

    python tools/e2e_sweep.py [--size 256] [--batches 16,64] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=256)
    p.add_argument("--batches", default="16,64")
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--modes", default="plain,bench,cl,bench_cl")
    args = p.parse_args()
    from bench import build_model
    from gdeconv.synth import make_batch
    dev = torch.device("cuda:0")
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    model = build_model(8, "Gaussian", dev)
    for mode in args.modes.split(","):
        torch.backends.cudnn.benchmark = "bench" in mode
        cl = "cl" in mode
        model.Z.to(memory_format=torch.channels_last if cl else torch.contiguous_format)
        for B in [int(b) for b in args.batches.split(",")]:
            obs, psf, alpha, _ = make_batch(B, args.size, seed=5, device=dev)
            with torch.no_grad():
                model(obs, psf, alpha)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.reps):
                    model(obs, psf, alpha)
                torch.cuda.synchronize()
                t = (time.perf_counter() - t0) / args.reps
                x = torch.rand(B, 1, args.size, args.size, device=dev)
                if cl:
                    x = x.contiguous(memory_format=torch.channels_last)
                model.Z(x)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                model.Z(x)
                torch.cuda.synchronize()
                tz = time.perf_counter() - t1
            print(json.dumps({"mode": mode, "batch": B, "size": args.size, "gal_per_s": B / t,
                              "denoiser_ms_per_call": tz * 1e3, "forward_ms": t * 1e3,
                              "denoiser_share": 8 * tz / t}), flush=True)
            del obs, psf, alpha, x
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
