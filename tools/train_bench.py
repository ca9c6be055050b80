"""Training-step throughput of UnrolledADMMGaussian (the model train.py:41 trains).

One step = forward of ``UnrolledADMMGaussian(n_iters=8, subnet=True)`` (HIP X update with its HIP
backward, PyTorch ResUNet nc=32..256 and SubNet in train mode) + MultiScaleLoss (L1 over 1x, 2x, 4x
average pools weighted 1, 1/2, 1/4 - utils/utils_train.py:256-284, restated) + backward + gradient
clipping at norm 1 + Adam (lr 1e-4) + loss.item(), as train.py:83-92 does.  Synthetic seeded batches (gdeconv.synth) of the reference's batch size 32
at 48^2, deterministic weights.  Prints one JSON line.

    python tools/train_bench.py [--batch 32] [--size 48] [--steps 10] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))


def multiscale_l1(out, tgt, scales=3):
    loss = 0.0
    for i in range(scales):
        k = 2 ** i
        o, t = (F.avg_pool2d(out, k, k), F.avg_pool2d(tgt, k, k)) if k > 1 else (out, tgt)
        loss = loss + F.l1_loss(o, t) / k
    return loss


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--size", type=int, default=48)
    p.add_argument("--n-iters", type=int, default=8)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    args = p.parse_args()
    from gdeconv.models import UnrolledADMMGaussian
    from gdeconv.synth import make_batch
    from gdeconv.weights import make_state_dict
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda:0")
    m = UnrolledADMMGaussian(n_iters=args.n_iters, subnet=True)
    m.load_state_dict(make_state_dict(m, 1234))
    m = m.to(dev).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    batches = [make_batch(args.batch, args.size, seed=100 + i, device=dev) for i in range(4)]

    def step(i):
        obs, psf, alpha, gt = batches[i % len(batches)]
        opt.zero_grad(set_to_none=True)
        out = m(obs, psf, alpha)
        loss = multiscale_l1(gt, out)                               # loss_fn(gt, rec), train.py:87
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)       # train.py:90
        opt.step()
        return loss.item()                                         # train.py:92 (a host sync per step)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    with torch.no_grad():
        m.eval()
        obs, psf, alpha, _ = batches[0]
        m(obs, psf, alpha)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            m(obs, psf, alpha)
        torch.cuda.synchronize()
        tf = time.perf_counter() - t1
    print(json.dumps({"metric": "UnrolledADMMGaussian training step", "batch": args.batch, "size": args.size,
                      "n_iters": args.n_iters, "train_galaxies_per_s": args.batch * args.steps / t,
                      "train_ms_per_step": t / args.steps * 1e3, "eval_forward_galaxies_per_s": args.batch * args.steps / tf,
                      "final_loss": float(loss), "dtype": "f32", "data": "synthetic (gdeconv.synth), deterministic weights"}))


if __name__ == "__main__":
    main()
