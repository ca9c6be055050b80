"""Placement probe for the 256^2 Gaussian iteration (k_gal_reg MID): time op_admm_iter with the state slots, z and
zin at controlled relative offsets inside ONE device allocation, eager and as a replayed hipGraph.

    python tools/placement_probe.py [--batch 4096] [--iters 24] [--blocks 3] > gpurun_out/placement.txt

Each configuration: one ADMMState, its state buffer and zin (and a separate z when not aliased) re-pointed into a
fresh arena at the given offsets, init, two warm iterations, then `blocks` x `iters` middle iterations timed with
HIP events (median block, ms per iteration).  The bench aliases z = zin (identity denoiser); the product path has z
in its own buffer (the ResUNet output).  Not part of the product: a measurement tool.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))

import torch  # noqa: E402

MB = 1 << 20
KB = 1 << 10


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--iters", type=int, default=24)
    p.add_argument("--blocks", type=int, default=3)
    p.add_argument("--only", default=None)
    args = p.parse_args()
    from gdeconv import engine
    from gdeconv.synth import make_batch
    dev = torch.device("cuda:0")
    N, L = args.batch, 256
    obs, psf, alpha, _ = make_batch(N, L, seed=20250307, device=dev)
    img = N * L * L * 4
    st0 = engine.ADMMState(obs, psf, alpha, "Gaussian")
    sbytes = st0.state.numel()
    del st0
    torch.cuda.synchronize()
    print(f"N={N}: state {sbytes / MB:.1f} MiB, image {img / MB:.1f} MiB", flush=True)
    r = engine.RhoSchedule(torch.ones(N, 1, 1, 4 + args.iters, device=dev), N, dev)

    def run(tag, zin_off, z_off, state_off, graph=False):
        """offsets in bytes inside one arena; z_off None: z aliases zin (the bench's identity denoiser)."""
        ends = [state_off + sbytes, zin_off + img] + ([z_off + img] if z_off is not None else [])
        arena = torch.empty(max(ends) + 4 * MB, dtype=torch.uint8, device=dev)
        base = arena.data_ptr()
        st = engine.ADMMState(obs, psf, alpha, "Gaussian")
        st.state = arena[state_off:state_off + sbytes]
        st.zin = arena[zin_off:zin_off + img].view(torch.float32).view(N, 1, L, L)
        st._fixed = (st._fixed[0], st._fixed[1], st._fixed[2], st.state.data_ptr(), st._fixed[4])
        st._bind()
        with torch.no_grad():
            st.init(None)
            z = st.zin if z_off is None else arena[z_off:z_off + img].view(torch.float32).view(N, 1, L, L)
            if z_off is not None:
                z.copy_(st.zin)
            st.step(z, r[0], r[0], r[1])           # FIRST
            st.step(z, r[1], r[1], r[2])
            times = []
            if graph:
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=side):
                    for i in range(args.iters):
                        st.step(z, r[2 + i], r[2 + i], r[3 + i])
                g.replay()
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(args.blocks):
                e0.record()
                if graph:
                    g.replay()
                else:
                    for i in range(args.iters):
                        st.step(z, r[2 + i], r[2 + i], r[3 + i])
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / args.iters)
        med = sorted(times)[len(times) // 2]
        print(f"{tag:44s} base%2MiB={base % (2 * MB) // KB:5d}K zin@{zin_off / MB:9.3f}M "
              f"z@{'alias' if z_off is None else f'{z_off / MB:.3f}M':>10s} state@{state_off / MB:8.3f}M "
              f"{'graph' if graph else 'eager'}  {med:.4f} ms/iter  blocks {[round(t, 4) for t in times]}", flush=True)
        del st, arena
        if graph:
            del g
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        return med

    S = sbytes
    cfgs = []
    # z aliased (bench): zin right after the state with several gaps
    for gap in (0, 256 * KB, 512 * KB, 1 * MB, 2 * MB, 2 * MB + 256 * KB, 64 * KB, 128 * KB):
        cfgs.append((f"alias gap {gap // KB}K", S + gap, None, 0))
    # zin first, state after
    for gap in (0, 256 * KB, 1 * MB):
        cfgs.append((f"alias zin-first gap {gap // KB}K", 0, None, img + gap))
    # distinct z (product path)
    for gap in (0, 256 * KB, 1 * MB):
        cfgs.append((f"distinct z gap {gap // KB}K", S + gap, S + gap + img + gap, 0))
    for c in cfgs:
        if args.only and args.only not in c[0]:
            continue
        run(*c)
        run(*c, graph=True)
        time.sleep(0.2)


if __name__ == "__main__":
    main()
