#!/usr/bin/env python3
"""Benchmark: unrolled PnP-ADMM spectral engine, galaxies/s at 256x256, n_iters=8 (BASELINE.json).

One "step" = one forward of the drop-in ``Unrolled_ADMM(n_iters=8, llh='Gaussian')`` over this
rank's batch (default 4096 galaxies of 256x256 fp32 = configs[2]; 8 ranks x 4096 = configs[3]):
SubNet (PyTorch) -> OTF + init_l2 -> 8 x [X-update / duals / V step] on the HIP engine, with the
denoiser replaced by the identity so the timed region is exactly the hot path the engine owns
(the ResUNet stays PyTorch per the north star; its end-to-end cost is reported separately as
``end_to_end`` on a sample).  Inputs are synthetic (``gdeconv.synth``), weights deterministic
(``gdeconv.weights``), all resident in HBM before timing.

  python bench.py [--gpus N --steps K --warmup W]

N > 1: under torch.distributed.run (WORLD_SIZE set) each process is one rank; without a launcher the
process spawns the N ranks itself (``spawn_ranks``) and forwards rank 0's line.  A process group whose
size is not N, or fewer visible GPUs than RCCL ranks, exits non-zero.

Rank 0 prints ONE JSON line (value = all ranks' galaxies / max-over-ranks wall time).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 TB/s measured float4 copy)
FP32_PEAK_TFLOPS = 157.3  # MI355X fp32 vector / MFMA peak (MI355X_MICROARCH.md)


def resunet_flops(L):
    """FLOPs of one ResUNet (models/ResUNet.py, nc = [64, 128, 256, 512], nb = 2) call on one L x L
    galaxy: 2 x MACs of every 3x3 / 2x2 convolution and transposed convolution (biases and ReLUs
    ignored).  141.9 GFLOP at 256^2."""
    nc, nb, tot = [64, 128, 256, 512], 2, 0
    def conv(cin, cout, k, hw):
        return 2 * cin * cout * k * k * hw
    hw = L * L
    tot += conv(1, nc[0], 3, hw)                                  # head
    for i in range(3):                                            # down: nb res blocks + strided 2x2
        tot += nb * 2 * conv(nc[i], nc[i], 3, hw)
        hw //= 4
        tot += conv(nc[i], nc[i + 1], 2, hw)
    tot += nb * 2 * conv(nc[3], nc[3], 3, hw)                     # body
    for i in (2, 1, 0):                                           # up: transposed 2x2 + nb res blocks
        hw *= 4
        tot += 2 * nc[i + 1] * nc[i] * hw                         # transposed 2x2 / 2: one tap per output
        tot += nb * 2 * conv(nc[i], nc[i], 3, hw)
    tot += conv(nc[0], 1, 3, hw)                                  # tail
    return tot

# kernel mode ids (gd_engine.hip enums) -> readable names
MODE_NAMES = {
    "k_row_fwd": ["ITER", "PSF_Y", "PSF_YP", "PSF_RAW", "PSF", "ONE", "TWO", "YA"],
    "k_col": ["ITER", "OTF_INIT", "OTF_CONV", "WIENER", "OTF", "CONV", "CONVC", "CONV2", "FWD", "INV",
              "G_INIT", "G_ITER", "G_W1", "G_ITER_F", "G_ITER_L", "G_ITER_FL"],
    "k_row_inv": ["ITER", "INIT", "OUT1", "OUT2", "RL_FINAL"],
    "k_row_invfwd": ["CLAMP", "RL_RATIO", "RL_UPDATE"],
    "k_subnet_features": ["FEATURES", "PSF"],
    "k_subnet_rhos": ["-", "-", "FUSED"],
    "k_subnet_mlp": ["MLP"],
    "k_gal_reg": ["MID", "FIRST", "LAST", "FIRST_LAST"],
    "k_gal_small": ["MID", "FIRST", "LAST", "FIRST_LAST"],
    "k_gal_init": ["-", "Y", "W1", "ONE", "REG", "POIS"],
    "k_pois_a": ["MID", "FIRST", "LAST", "FIRST_LAST"],
    "k_pois_b": ["ITER", "INIT"],
    "k_psf_rows": ["ROWS", "STATE"],
}
# fused Gaussian iteration / init implementations (gd_set_fused_iteration / gd_set_fused_init)
ITER_IMPL = {1: "k_gal_reg (512 threads, nothing parked in global memory)"}
INIT_IMPL = {1: "k_psf_rows + k_gal_reg_init (one launch)"}


def pretty(name):
    k, rest = name.split("<")
    L, mode = rest.rstrip(">").split(",")
    if k == "op_rl":
        return f"op_richardson_lucy<{L}>"
    if k.startswith("op_"):
        return f"{k}<{L},{['Gaussian', 'Poisson'][int(mode)]}>"
    names = MODE_NAMES.get(k)
    return f"{k}<{L},{names[int(mode)]}>" if names and int(mode) < len(names) else name


def op_bytes(name, L, n_iters, fused=False, h=48):
    """Compulsory (algorithmic) HBM bytes per galaxy of one call of a whole engine operation: every
    input the operation needs read once, every output written once, averaged
    over the first / middle / last ADMM iteration.  This is the roofline model of every bench line;
    the PMC 'traffic' field is what the kernels actually move.
      op_admm_iter, Gaussian, fused (k_gal_reg, k_gal_small): z + |H|^2, G, U1, W~ in, U1, W~ + zin out
        = 2 img + 5.5 half (first: no U1 read, 4.5; last: no G read, nothing written, 2.5; first-and-last
        at 256^2 reads G to form W~1, 2.5); three-kernel: + the RF / C / RI workspace round trips.
      op_admm_init, Gaussian, fused: y + PSF in, |H|^2, G, W~ (or F(x0)) + zin out = 2 img + 2.5 half
        + the PSF (h^2 floats) and at 256^2 its compact row spectra (h (L/2 + 1) complex, written and read; at
        160^2 the packed row-pair spectra, h/2 x L complex).
      op_admm_init, Poisson, 256^2 two-pass: 4 img + 5 half + the PSF and its compact rows (below)."""
    img, half, n = L * L * 4, (L // 2 + 1) * L * 8, max(1, n_iters)
    k = pretty(name)
    if k == f"op_richardson_lucy<{L}>":
        return survey_rl_bytes_per_galaxy(L, n_iters)
    if k == f"op_admm_iter<{L},Gaussian>":
        if n == 1:
            c = 2.5 if fused else 5.5
        elif fused:
            c = (4.5 + 5.5 * (n - 2) + 2.5) / n
        else:
            c = (2 + 6.5 + (2 + 7.5) * (n - 2) + 2 + 4.5) / n
        return 2 * img + c * half
    if k == f"op_admm_init<{L},Gaussian>" and fused:
        # k_psf_rows<STATE>'s compact row spectra [kx][i] (h (L/2 + 1) complex), written once and read once; the
        # round-3 model counted them twice over (5.70 GB at 4096 x 256^2 against PMC 5.32 GB = 0.93x; now 5.30 GB)
        # (160^2, k_gal_mid_init: the PSF's packed row-pair spectra [L][h/2] parked in the U1 slot, written and read)
        rows = 2 * h * (L // 2 + 1) * 8 if L == 256 else (2 * (h // 2) * L * 8 if L in (80, 96, 112, 128, 144, 160) else 0)
        return 2 * img + 2.5 * half + 4 * h * h + rows
    if k == f"op_admm_init<{L},Poisson>" and fused and L == 256:
        # two-pass Poisson init: k_psf_rows<STATE> (the PSF in, its compact row spectra out), k_gal_reg_init<POIS>
        # (y, the rows in; H -> G slot, zin out, H F(x0) -> W slot, H re-read for that product: 2 img + 3 half),
        # k_pois_b<INIT> (H F(x0), y in; w1 out, F(w1) -> W slot: 2 img + 2 half)
        rows = 2 * h * (L // 2 + 1) * 8
        return 4 * img + 5 * half + 4 * h * h + rows
    if k == f"op_admm_iter<{L},Poisson>":
        if fused and L == 256:
            # two-pass (gd_poisreg.hpp): pass A z, H, U1, W in, U1, H X, zin out (2 img + 5 half; first 4: no
            # U1; last 2 img + 3 half: nothing but x written); pass B H X, y, w in, w, F(w') out (3 img + 2 half)
            if n == 1:
                return 2 * img + 2 * half
            mid, first, last = 5 * img + 7 * half, 5 * img + 6 * half, 2 * img + 3 * half
            return (first + mid * (n - 2) + last) / n
        if fused and L <= 112:
            # k_pois_small: z, u1, w, y and the OTF in; u1, w, zin out (last: z, u1, w, OTF in, x alpha out)
            mid, last = 7 * img + half, 4 * img + half
            return (mid * (n - 1) + last) / n
        # u1, w (= v - u2), z in; u1, w, zin out (+ y, the OTF half spectrum); the last iteration
        # reads z, u1, w, y, OTF and writes x only
        mid, last = 6 * img + 2 * half, 4 * img + half
        return (mid * (n - 1) + last) / n
    return None


def kernel_bytes(name, L, n_iters):
    """Algorithmic HBM bytes per galaxy for one launch of a kernel (each compulsory input read once,
    each output written once), averaged over the launches of one forward where
    the first / last ADMM iteration moves less."""
    img = L * L * 4                  # one fp32 image
    half = (L // 2 + 1) * L * 8      # one complex64 half spectrum
    n = max(1, n_iters)
    k = pretty(name)
    table = {
        # Gaussian (spectral state |H|^2, G = conj(H)F(y/a), U1, W~ = conj(H)W): RF(z) -> C_G_ITER -> RI(zin)
        f"k_row_fwd<{L},ONE>": img + half,                                  # z -> T
        f"k_col<{L},G_ITER>": half * 7.5,                                   # T, |H|^2, G, U1, W~ -> U1, W~, T
        f"k_col<{L},G_ITER_F>": half * 6.5,                                 # T, |H|^2, G, W~ -> U1, W~, T
        f"k_col<{L},G_ITER_L>": half * 4.5,                                 # T, |H|^2, U1, W~ -> T
        f"k_col<{L},G_W1>": half * 3.5,                                     # x0 T, |H|^2, G -> W~
        f"k_gal_reg<{L},MID>": 2 * img + 5.5 * half,                        # z, |H|^2, G, U1, W~ -> U1, W~, zin
        f"k_gal_reg<{L},FIRST>": 2 * img + 4.5 * half,
        f"k_gal_reg<{L},LAST>": 2 * img + 2.5 * half,
        f"k_row_inv<{L},OUT1>": half + img,                                 # T -> zin | x
        f"k_row_fwd<{L},YA>": img + half,                                   # y -> T
        f"k_col<{L},G_INIT>": half + 2.5 * half,                            # T -> |H|^2, G, T (PSF: 9 KB)
        # Poisson (spatial u1, w): RF(z-u1, w) -> C_ITER -> RI_ITER
        f"k_row_fwd<{L},ITER>": 3 * img + 2 * half,
        f"k_col<{L},ITER>": 5 * half,
        f"k_row_inv<{L},ITER>": ((2 * half + 7 * img) * (n - 1) + (2 * half + img)) / n,
        f"k_col<{L},OTF_INIT>": 4 * half,
        f"k_col<{L},CONV>": 3 * half,
        f"k_row_inv<{L},INIT>": half + 3 * img,
        # shared setup
        f"k_row_fwd<{L},PSF_Y>": img + 2 * half,                            # y (+ 9 KB PSF) -> T(2)
        f"k_row_invfwd<{L},CLAMP>": 2 * half + img,                         # T -> zin, T
    }
    return table.get(k)


def graph_iter_ms(obs, psf, alpha, dev, reps=64, llh="Gaussian"):
    """Average device time of one middle ADMM iteration (gd_admm_iter) without host gaps: ``reps`` launches on
    one state, z fixed, captured in a hipGraph and replayed between two HIP events."""
    from gdeconv import engine
    N = obs.shape[0]
    with torch.no_grad():
        st = engine.ADMMState(obs, psf, alpha, llh)
        r = engine.RhoSchedule(torch.ones(N, 1, 1, reps + 2, device=dev), N, dev)
        st.init(r[0] if st.init_reads_rho else None)
        z = st.zin.clone()
        st.step(z, r[0], r[0], r[1])  # iteration 0 (FIRST) outside the graph
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            for i in range(1, reps + 1):
                st.step(z, r[i], r[i], r[i + 1])
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times = []
        for _ in range(5):  # the median of 5 replays (one replay is ~0.4 ms: a single sample was noisy)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / reps)
        return sorted(times)[len(times) // 2]


def survey_bytes_per_galaxy(L, n, h=48):
    """B = 4*HW*(4 + 16 n) + 4 h w (ADMM spectral engine, per galaxy)."""
    return 4 * L * L * (4 + 16 * n) + 4 * h * h


def survey_rl_bytes_per_galaxy(L, n, h=48):
    """Richardson-Lucy B = 4*HW*(3 + 4 n) + 4 h w per galaxy (per iteration: read x, y,
    the OTF, write x)."""
    return 4 * L * L * (3 + 4 * n) + 4 * h * h


class RLForward(torch.nn.Module):
    """``Richard_Lucy(n_iters).forward(y, psf)`` behind the (y, psf, alpha) call of the ADMM bench."""

    def __init__(self, n_iters):
        super().__init__()
        from gdeconv.models import Richard_Lucy
        self.rl = Richard_Lucy(n_iters)

    def forward(self, y, psf, alpha=None):
        return self.rl(y, psf)


def progress(msg):
    """A progress line on stderr (the JSON result goes to stdout alone)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--blocks", type=int, default=3, help="timed blocks of --steps steps (value = the median block)")
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=4096, help="galaxies per GPU")
    p.add_argument("--size", type=int, default=256)
    p.add_argument("--n-iters", type=int, default=None, help="default 8 (admm) / 100 (rl)")
    p.add_argument("--workload", choices=["admm", "rl"], default="admm",
                   help="admm: Unrolled_ADMM (BASELINE metric, configs[2]); rl: Richard_Lucy (configs[4])")
    p.add_argument("--llh", default="Gaussian")
    p.add_argument("--cpu-sample", type=int, default=64, help="galaxies in the CPU baseline sample")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--e2e-sample", type=int, default=512, help="galaxies for the ResUNet end-to-end sample")
    p.add_argument("--e2e-forwards", type=int, default=2, help="timed forwards of the end-to-end sample")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--no-graph", action="store_true", help="skip the hipGraph-replay measurement")
    p.add_argument("--no-ingest", action="store_true", help="skip the packed-file ingest pipeline measurement")
    p.add_argument("--ingest-dir", default=None, help="where the ingest measurement writes its packed file")
    p.add_argument("--chunk-mb", type=float, default=None,
                   help="Infinity-Cache chunk working set in MiB (0 = off; default: library default)")
    p.add_argument("--pipe-streams", type=int, default=None, help="internal HIP streams for chunk pipelining")
    p.add_argument("--fused-init", type=int, default=None,
                   help="Gaussian init: 1 the one-launch kernels (256^2: k_psf_rows + k_gal_reg_init), 0 the chunked chain")
    p.add_argument("--fused", type=int, default=None,
                   help="iterations: 1 the one-launch kernels (256^2: k_gal_reg), 0 the chained path")
    p.add_argument("--fused-rl", type=int, default=None,
                   help="Richardson-Lucy at 256^2: 1 k_rl_reg (the whole loop per galaxy), 0 the chunked chain")
    p.add_argument("--settle-s", type=float, default=2.0,
                   help="after the warmup steps, untimed steps until this many seconds of load (clock settling)")
    p.add_argument("--no-extra", action="store_true",
                   help="default run only: skip the configs[1] / configs[4] sub-lines")
    p.add_argument("--traffic-json", default=None,
                   help="rocprofv3 --pmc summary (per-kernel HBM bytes) for the roofline 'traffic' field "
                        "(default: profiles/pmc_traffic.json, _48 / _rl variants for those workloads)")
    return p.parse_args()


def build_model(n_iters, llh, dev, seed=1234):
    from gdeconv.models import Unrolled_ADMM
    from gdeconv.weights import make_state_dict
    m = Unrolled_ADMM(n_iters=n_iters, llh=llh)
    m.load_state_dict(make_state_dict(m, seed))
    return m.to(dev).eval()


def cpu_baseline(args):
    """The oracle (PyTorch CPU restatement of the reference) on a bounded sample of the same
    workload: same model config, denoiser = identity, SubNet rhos from the same weights."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import admm_oracle as O
    from gdeconv.synth import make_batch
    n = args.cpu_sample
    obs, psf, alpha, _ = make_batch(n, args.size, seed=777)
    if args.workload == "rl":
        O.richardson_lucy(obs[:1], psf[:1], 2)  # warm
        t_total, done = 0.0, 0
        while t_total < args.cpu_seconds or done == 0:
            t0 = time.perf_counter()
            O.richardson_lucy(obs, psf, args.n_iters)
            t_total += time.perf_counter() - t0
            done += n
        return {"value": done / t_total, "unit": "galaxies/s", "cores": torch.get_num_threads(), "kind": "port",
                "sample": f"oracle/admm_oracle.richardson_lucy (PyTorch CPU restatement of the reference), "
                          f"{n} galaxies x {args.size}^2, n_iters={args.n_iters}, {done // n} passes, {t_total:.1f}s"}
    m = build_model(args.n_iters, args.llh, "cpu")
    with torch.no_grad():
        rho1, rho2 = m.init(psf, alpha)
        t_total, done = 0.0, 0
        O.admm_forward(obs[:2], psf[:2], alpha[:2], rho1[:2], rho2[:2], args.llh)  # warm
        while t_total < args.cpu_seconds or done == 0:
            t0 = time.perf_counter()
            O.admm_forward(obs, psf, alpha, rho1, rho2, args.llh)
            t_total += time.perf_counter() - t0
            done += n
    return {"value": done / t_total, "unit": "galaxies/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle/admm_oracle.admm_forward (PyTorch CPU restatement of the reference), "
                      f"{n} galaxies x {args.size}^2, n_iters={args.n_iters}, {args.llh}, denoiser=identity, "
                      f"{done // n} passes, {t_total:.1f}s"}


def spawn_ranks(args, argv):
    """``--gpus N > 1`` without a launcher: start N fresh rank processes through
    ``torch.distributed.run`` (127.0.0.1, a free port) as CHILDREN of this process - which has made no
    GPU call (no torch.cuda.*, no engine library) and never execs - forward rank 0's JSON line to
    stdout, and return the launcher's exit code (non-zero also when no line came back)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    print(f"[bench] --gpus {args.gpus} without WORLD_SIZE: launching {args.gpus} ranks: {' '.join(cmd)}",
          file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    line = None
    for ln in proc.stdout:
        s = ln.strip()
        if s.startswith("{") and '"metric"' in s:
            line = s
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if line is not None:
        print(line, flush=True)
    if rc == 0 and line is None:
        print("[bench] error: the ranks exited without a result line", file=sys.stderr)
        rc = 1
    return rc


def all_ranks(x, world, backend, dev):
    """A host float from every rank (all_gather; on the device under RCCL, in host memory under gloo)."""
    if world == 1:
        return [float(x)]
    d = dev if backend == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=d)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def max_over_ranks(x, world, backend, dev):
    """MAX of a host float over the ranks (on the device under RCCL, in host memory under gloo)."""
    if world == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args, sys.argv[1:]))
    from gdeconv import _lib
    from gdeconv.dist import init_process_group, local_device

    rank, world, local = init_process_group()
    if world != args.gpus:
        print(f"[bench] error: --gpus {args.gpus} but the process group has {world} rank(s) "
              f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')})", file=sys.stderr)
        sys.exit(2)
    backend = dist.get_backend() if world > 1 else None
    if backend == "nccl" and torch.cuda.device_count() < world:
        print(f"[bench] error: {world} RCCL ranks but {torch.cuda.device_count()} visible GPU(s)", file=sys.stderr)
        sys.exit(2)
    dev = local_device(local)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    lib = _lib.load()
    ctx = {"lib": lib, "rank": rank, "world": world, "backend": backend, "dev": dev}
    rec = measure(args, ctx)
    # the other BASELINE configs a single GPU runs, as sub-lines of the default run (each with its own
    # step count, roofline and CPU baseline): configs[1] (256 x 48^2) and configs[4] (RL(100), 4096 x 256^2)
    if world == 1 and not args.no_extra and args.workload == "admm" and args.size == 256 and args.llh == "Gaussian":
        for key, over in (("configs1", dict(batch=256, size=48, n_iters=8, steps=max(200, args.steps),
                                            warmup=max(20, args.warmup), settle_s=0.5, no_ingest=True,
                                            e2e_sample=256, e2e_forwards=max(10, args.e2e_forwards),
                                            cpu_sample=64)),
                          ("configs4", dict(workload="rl", batch=4096, size=256, n_iters=100, steps=args.steps,
                                            warmup=min(2, args.warmup), settle_s=1.0, no_ingest=True, no_e2e=True,
                                            no_graph=True, cpu_sample=4))):
            sub = argparse.Namespace(**{**vars(args), **over, "traffic_json": None})
            torch.cuda.empty_cache()
            rec[key] = measure(sub, ctx)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


def measure(args, ctx):
    """One workload (args.workload / size / batch / n_iters / llh) on this rank: warm-up, clock settling, the
    timed K steps, the profiling pass, and the fields beside value.  Returns the record (rank 0's is printed)."""
    from gdeconv import _lib
    from gdeconv.synth import make_batch
    lib, rank, world, backend, dev = ctx["lib"], ctx["rank"], ctx["world"], ctx["backend"], ctx["dev"]
    if args.chunk_mb is not None:
        lib.gd_set_chunk_bytes(int(args.chunk_mb * (1 << 20)))
    chunk_bytes = lib.gd_set_chunk_bytes(0)
    lib.gd_set_chunk_bytes(chunk_bytes)
    if args.fused is not None:
        lib.gd_set_fused_iteration(args.fused)
    if args.fused_init is not None:
        lib.gd_set_fused_init(args.fused_init)
    if args.fused_rl is not None:
        lib.gd_set_fused_rl(args.fused_rl)
    fused_init = lib.gd_set_fused_init(1)
    lib.gd_set_fused_init(fused_init)
    fused = lib.gd_set_fused_iteration(0)
    lib.gd_set_fused_iteration(fused)
    generic = args.size not in (32, 48, 64, 96, 128, 256)  # gd_supported_size == 2: gd_generic.hpp
    # 80 / 112 / 144 / 160 (runtime-planned sizes) and 96 / 128 run their Gaussian iterations and init fused too
    # (k_gal_mid, k_gal_mid_init: gd_engine.hip mid_size, GD_MID_EXTRA)
    mid_fused = bool(fused) and args.size in (80, 96, 112, 128, 144, 160) and args.llh == "Gaussian"
    # 256^2 Gaussian batches below gd_set_fused_min_batch run the chained kernels (one-workgroup-per-galaxy launches
    # of fewer than ~a round of workgroups leave most CUs idle)
    min_batch = lib.gd_set_fused_min_batch(0, -1)
    small_chained = args.size == 256 and args.llh == "Gaussian" and args.batch < min_batch
    use_fused = bool(fused) and (not generic or mid_fused) and args.llh == "Gaussian" and not small_chained
    if small_chained:
        fused_init = 0
    pois2 = (bool(fused) and args.size == 256 and args.llh == "Poisson"  # two whole-galaxy passes per iteration
             and args.batch >= lib.gd_set_fused_min_batch(1, -1))
    # Poisson at L <= 112: one workgroup per galaxy, both images in LDS (k_pois_small, k_pois_small_init)
    pois_small = bool(fused) and args.llh == "Poisson" and args.size in (32, 48, 64, 80, 96, 112)
    if args.pipe_streams is not None:
        lib.gd_set_pipeline_streams(args.pipe_streams)
    pipe_streams = lib.gd_set_pipeline_streams(0)

    rl = args.workload == "rl"
    if args.n_iters is None:
        args.n_iters = 100 if rl else 8
    if rl and args.cpu_sample == 64:
        args.cpu_sample = 4                  # RL(100) on the CPU: ~1 s per 256^2 galaxy
    N, L, n = args.batch, args.size, args.n_iters
    obs, psf, alpha, _ = make_batch(N, L, seed=20250307 + rank, device=dev)
    if rl:
        model, denoiser = RLForward(n).to(dev), None
        use_fused = False
        fused_rl = lib.gd_set_fused_rl(1)
        lib.gd_set_fused_rl(fused_rl)
        fused_rl = fused_rl and N >= lib.gd_set_fused_min_batch(2, -1)   # small batches: the chunked chain
        rl_impl = ("fused, k_rl_reg (OTF, then each galaxy's whole loop in one 512-thread workgroup; x, y, OTF "
                   "re-read from the Infinity Cache)" if (fused_rl and L == 256) else
                   "whole RL loop per Infinity-Cache chunk (RIF/C chain)")
    else:
        model = build_model(n, args.llh, dev)
        denoiser = model.Z
        model.Z = torch.nn.Identity()        # spectral engine: the HIP hot path

    def step():
        return model(obs, psf, alpha)

    progress(f"{args.workload} {N} x {L}^2 n_iters={n}: warm-up")
    with torch.no_grad():
        for _ in range(args.warmup):
            out = step()
        torch.cuda.synchronize()
        # clock settling: the chip's clocks and HBM rate drift for the first ~second of sustained load (round 4:
        # value 312.8 k against 296 k in the same run's later interleaved blocks), so more untimed steps run
        # until --settle-s seconds of this workload have passed; reported as clock_settle, apart from warmup
        ts, settle = time.perf_counter(), 0
        while time.perf_counter() - ts < args.settle_s:
            out = step()
            settle += 1
            if settle % 4 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        settle_s = time.perf_counter() - ts
        # the hipGraph of the same forward (gdeconv.graphs), captured before the timed blocks so that its replayed
        # blocks interleave with the eager ones in one clock window: what a serving loop pays once host launch
        # overhead is gone (matters at 48^2; reported beside value, not as value)
        gf = None
        if not args.no_graph:
            progress("hipGraph capture")
            from gdeconv.graphs import GraphedForward
            gf = GraphedForward(model, obs, psf, alpha)
            gout = gf.replay()
            torch.cuda.synchronize()

        def timed(fn, prof=0):
            """K steps of fn bracketed by a barrier + synchronize on both sides; max over ranks (seconds)."""
            if world > 1:
                dist.barrier()
            if prof:
                _lib.profile_enable(prof)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.steps):
                r = fn()
            torch.cuda.synchronize()
            t = time.perf_counter() - t
            if prof:
                _lib.profile_enable(0)
            return max_over_ranks(t, world, backend, dev), r

        # B timed blocks of exactly K steps each; after every eager block (no profiling events: value's blocks) the
        # same window runs K replayed steps (if graphed) and K steps with the library's HIP events on (per operation
        # on the caller's stream, per launch too when nothing is pipelined: the roofline's launch durations).
        # value = the MEDIAN eager block; every block is recorded.
        _lib.profile_enable(0)
        _lib.profile_reset()
        prof_level = 1 if chunk_bytes > 0 else 2
        te_blocks, tg_blocks, tp_blocks, rank_blocks = [], [], [], []
        for _ in range(args.blocks):
            t_, out = timed(step)
            te_blocks.append(t_)
            rank_blocks.append(all_ranks(t_, world, backend, dev) if world > 1 else [t_])
            if gf is not None:
                t_, gout = timed(gf.replay)
                tg_blocks.append(t_)
            tp_blocks.append(timed(step, prof_level)[0])
        kstats = _lib.profile_collect()
        assert torch.isfinite(out).all(), "non-finite output"

    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
    elapsed = med(te_blocks)
    tp = med(tp_blocks)
    progress(f"eager blocks {[round(t * 1e3 / args.steps, 3) for t in te_blocks]} ms/step; replayed "
             f"{[round(t * 1e3 / args.steps, 3) for t in tg_blocks]}; profiled {[round(t * 1e3 / args.steps, 3) for t in tp_blocks]}")
    rank_times = rank_blocks[te_blocks.index(elapsed)]
    gal_s = N * world * args.steps / elapsed

    gather_ms, with_gather = None, None
    if world > 1:
        # the optional final collection over xGMI (RCCL all_gather_into_tensor), timed on its own ...
        from gdeconv.dist import gather_batch
        torch.cuda.synchronize()
        dist.barrier()
        tg = time.perf_counter()
        gather_batch(out, N * world)
        torch.cuda.synchronize()
        gather_ms = max_over_ranks(time.perf_counter() - tg, world, backend, dev) * 1e3
        gathered_bytes = N * world * out[0].numel() * out.element_size()   # the [N * world, 1, H, W] result
        # ... and overlapped: step k's gather in flight (RCCL's stream) while step k + 1 computes
        with torch.no_grad():
            dist.barrier()
            torch.cuda.synchronize()
            tw = time.perf_counter()
            pend = None
            for _ in range(args.steps):
                o_ = step()
                if pend is not None:
                    pend.wait()
                pend = gather_batch(o_, N * world, async_op=True)
            pend.wait()
            torch.cuda.synchronize()
            tw = max_over_ranks(time.perf_counter() - tw, world, backend, dev)
        with_gather = {"value": N * world * args.steps / tw, "unit": "galaxies/s",
                       "ms_per_step": tw * 1e3 / args.steps,
                       "note": "each step's outputs all-gathered to every rank, overlapped with the next step"}

    graphed = None
    if gf is not None:
        tgr = med(tg_blocks)
        graphed = {"value": N * world * args.steps / tgr, "unit": "galaxies/s", "ms_per_step": tgr * 1e3 / args.steps,
                   "note": "median of the replayed blocks interleaved with value's eager blocks (no per-op profiling events)",
                   "bit_identical_to_eager": bool(torch.equal(gout, out))}
        del gf, gout

    # host ingest (gdeconv.ingest): the same batch written once to a GDPACK01 file, then K steps of
    # {native pread -> pinned slot -> H2D on a copy stream -> forward}, prefetching one batch ahead:
    # the PCIe-inclusive rate from a file in the page cache (reported beside value, never as value)
    ingest = None
    if not args.no_ingest:
        progress("packed-file ingest pipeline")
        import tempfile
        from gdeconv.ingest import DeviceBatches, PackedGalaxies, write_pack
        idir = args.ingest_dir or tempfile.gettempdir()
        ipath = os.path.join(idir, f"gd_bench_{os.getpid()}_{rank}.gdpack")
        try:
            write_pack(ipath, obs.cpu(), psf.cpu(), alpha=alpha.reshape(-1).cpu().numpy())
            nthr = min(16, os.cpu_count() or 1)
            with PackedGalaxies(ipath, threads=nthr) as pk, torch.no_grad():
                order = np.tile(np.arange(N), args.steps + 1)
                it = iter(DeviceBatches(pk, N, dev, indices=order))
                o_, p_, a_ = next(it)   # warm (first slot fill + pinned allocation)
                iout = model(o_, p_, a_)
                torch.cuda.synchronize()
                if world > 1:
                    dist.barrier()
                ti0 = time.perf_counter()
                for o_, p_, a_ in it:
                    iout = model(o_, p_, a_)
                torch.cuda.synchronize()
                ti = max_over_ranks(time.perf_counter() - ti0, world, backend, dev)
                per_gal = (L * L + psf.shape[-1] * psf.shape[-2] + 1) * 4
                ingest = {"value": N * world * args.steps / ti, "unit": "galaxies/s", "ms_per_step": ti * 1e3 / args.steps,
                          "bytes_per_galaxy": per_gal, "host_to_device_GBs": per_gal * N * args.steps / ti / 1e9,
                          "reader_threads": nthr, "bit_identical_to_resident": bool(torch.equal(iout, out)),
                          "sample": f"{N} galaxies/GPU from a GDPACK01 file in the page cache ({idir}), "
                                    "one batch prefetched ahead, identity denoiser"}
        finally:
            if os.path.exists(ipath):
                os.remove(ipath)

    # live timing: HIP events recorded by the library on each kernel's launch stream and, for whole
    # operations (op_*), on the caller's stream, over the timed region
    kernels = {pretty(k): {"avg_ms": ms / c, "launches": c} for k, (ms, c) in kstats.items()}
    ops = {k: v for k, v in kstats.items() if k.startswith("op_")}
    kern = {k: v for k, v in kstats.items() if not k.startswith("op_")}
    pipelined = chunk_bytes > 0
    h_psf = psf.shape[-1]
    priced_ops = {k: v for k, v in ops.items() if op_bytes(k, L, n, use_fused or pois2 or pois_small, h_psf)}
    # every priced operation against the HBM spec (compulsory bytes / average call time)
    for k, (ms, c) in ops.items():
        b = op_bytes(k, L, n, use_fused or pois2 or pois_small, h_psf)
        if b:
            ach = b * N / (ms / c * 1e-3) / 1e9
            kernels[pretty(k)].update({"algorithmic_bytes_per_call": b * N, "achieved_GBs": ach,
                                       "frac_of_hbm_peak": ach / HBM_PEAK_GBS})
    if (pipelined or use_fused or pois2 or pois_small) and priced_ops:
        # chunks of RF -> C -> RI run concurrently on several streams: the roofline unit is the
        # whole ADMM iteration (one op_admm_iter call), timed on the caller's stream
        dom_raw = max(priced_ops, key=lambda k: ops[k][0])
        dom_ms = ops[dom_raw][0] / ops[dom_raw][1]
        per_gal = op_bytes(dom_raw, L, n, use_fused or pois2 or pois_small, h_psf)
    else:
        priced = {k: v for k, v in kern.items() if kernel_bytes(k, L, n)} or kern
        dom_raw = max(priced, key=lambda k: kern[k][0])
        dom_ms = kern[dom_raw][0] / kern[dom_raw][1]
        per_gal = kernel_bytes(dom_raw, L, n)
    timing = "HIP events on the caller's stream around each call, the profiled blocks interleaved with value's blocks"
    if (not rl and dom_ms < 0.05 and pretty(dom_raw) == f"op_admm_iter<{L},{args.llh}>"):
        # a short op of a host-bound eager forward (48^2): the events also time the host's enqueue gaps, so
        # the launch duration comes from back-to-back launches replayed as one hipGraph instead
        dom_ms = graph_iter_ms(obs, psf, alpha, dev, llh=args.llh)
        timing = "64 back-to-back middle iterations (gd_admm_iter) replayed as one hipGraph, HIP events around it, median of 5 replays"
    achieved = per_gal * N / (dom_ms * 1e-3) / 1e9 if per_gal else None
    traffic = None
    if args.traffic_json is None:
        suffix = "_rl" if rl else ("_poisson" if args.llh == "Poisson" else "") + ("" if L == 256 else f"_{L}")
        args.traffic_json = os.path.join(ROOT, "profiles", f"pmc_traffic{suffix}.json")
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        same_engine = tj.get("engine_rev") == lib.gd_engine_rev().decode()
        if same_engine and tj.get("batch") == N and tj.get("size") == L and tj.get("n_iters", n) == n:
            ent = tj.get("kernels", {}).get(pretty(dom_raw))
            traffic = ent.get("hbm_bytes_per_launch") if ent else None
            for k, v in kernels.items():  # PMC bytes per call beside every priced operation
                e = tj.get("kernels", {}).get(k)
                if e and "algorithmic_bytes_per_call" in v:
                    v["pmc_traffic_per_call"] = e.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    roofline = {"bound": "hbm", "kernel": pretty(dom_raw), "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic, "algorithmic_bytes_per_launch": per_gal * N if per_gal else None,
                "avg_launch_ms": dom_ms, "timing": timing}
    survey_b = survey_rl_bytes_per_galaxy(L, n) if rl else survey_bytes_per_galaxy(L, n)
    if rl:
        metric = f"galaxies/sec ({L}x{L}, Richard_Lucy n_iters={n})"
        workload = (f"Richard_Lucy(n_iters={n}) forward (OTF + {n} multiplicative FFT-conv iterations), "
                    f"batch {N}/GPU, {L}x{L} fp32" + (" (BASELINE.json configs[4])" if L == 256 and n == 100 else ""))
    else:
        metric = f"galaxies/sec ({L}x{L}, n_iters={n}) - unrolled ADMM spectral engine"
        workload = (f"Unrolled_ADMM(n_iters={n}, llh='{args.llh}') forward, denoiser=identity "
                    f"(spectral engine: SubNet + OTF + init_l2 + {n} ADMM iterations), "
                    f"batch {N}/GPU, {L}x{L} fp32" + (" (BASELINE.json configs[2]/[3])" if L == 256 else
                                                      " (BASELINE.json configs[1])" if L == 48 else
                                                      " (not a BASELINE config: runtime-planned size)" if generic
                                                      else " (not a BASELINE config)"))

    rec = {
        "metric": metric,
        "value": gal_s, "unit": "galaxies/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "clock_settle": {"steps": settle, "seconds": settle_s,
                                                "note": "untimed steps after the warmup steps, until --settle-s "
                                                        "seconds of sustained load had passed"},
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (gdeconv.synth, seeded); deterministic random weights (gdeconv.weights)",
        "config": {"workload": workload,
                   "global_batch": N * world, "image": [L, L], "psf": [48, 48], "n_iters": n,
                   "llh": None if rl else args.llh,
                   "parallelism": f"dp{world} (batch shards, no data-path collective"
                                  + (f"; {backend} process group, {world} ranks)" if backend else ")"),
                   "ranks_seen": world, "backend": backend or "none",
                   "chunk_mib": chunk_bytes / (1 << 20), "pipeline_streams": pipe_streams if pipelined else 1,
                   "iteration": (("fused, " + (ITER_IMPL[fused] if L == 256 else
                                               f"k_gal_mid ({L}^2: half spectrum in LDS, {256 if L <= 112 else 512} threads per galaxy)"
                                               if mid_fused else
                                               "k_gal_small (half spectrum in LDS, one workgroup per galaxy)"))
                                 if use_fused else (rl_impl if rl else
                                                    ("two whole-galaxy passes: k_gal_reg<POIS> (X update, u1, zin) + "
                                                     "k_pois_b (Hx, V step, duals, conj(H) F(w))") if pois2
                                                    else (f"fused, k_pois_small ({L}^2: both images in LDS, one workgroup "
                                                          "per galaxy)") if pois_small
                                                    else "three-kernel, runtime-planned line FFTs (gd_generic.hpp)"
                                                    if generic else
                                                    f"three-kernel (batch below gd_set_fused_min_batch = {min_batch})"
                                                    if small_chained else "three-kernel")),
                   "init": (None if rl else
                            ("fused, " + INIT_IMPL[fused_init] if fused_init else "chunked")
                            if (L == 256 and args.llh == "Gaussian") else
                            (("k_psf_rows + k_gal_reg_init<POIS>" if fused_init else "chunked Gaussian chain")
                             + " + k_pois_b<INIT>") if pois2 else
                            ("fused, k_gal_small_init (one launch)" if L <= 64 and args.llh == "Gaussian" and fused
                             and not generic else
                             f"fused, k_gal_mid_init ({L}^2: one launch, half spectrum in LDS)" if mid_fused and fused_init
                             else f"fused, k_pois_small_init ({L}^2: one launch, both images in LDS)"
                             if pois_small and fused_init
                             else "chunked" + (", runtime-planned line FFTs" if generic else "")))},
        "roofline": roofline,
        # SURVEY.md 8(d)'s per-galaxy byte model prices the reference's op-for-op path (16 fp32 words per
        # pixel per iteration); this engine's compulsory traffic is 7.5 (roofline above), so the survey
        # model is reported as a reference figure only, with no fraction of peak
        "reference_op_model": {"survey_bytes_per_galaxy": survey_b,
                               "note": "SURVEY 8(d) byte model of the reference's per-iteration FFT round trips; "
                                       "not this engine's traffic (see roofline / kernels.*.algorithmic_bytes_per_call)"},
        "kernels": kernels,
    }
    rec["blocks"] = {"eager_ms_per_step": [round(t * 1e3 / args.steps, 4) for t in te_blocks],
                     "graphed_ms_per_step": [round(t * 1e3 / args.steps, 4) for t in tg_blocks],
                     "profiled_ms_per_step": [round(t * 1e3 / args.steps, 4) for t in tp_blocks],
                     "eager_spread": max(te_blocks) / min(te_blocks) - 1.0,
                     "value_vs_profiled": gal_s / (N * world * args.steps / tp) - 1.0,
                     "note": f"{args.blocks} rounds of [K eager steps, K replayed steps, K profiled steps] after the "
                             "warmup and clock settling; value and ms_per_step = the median eager block; kernels.* and "
                             "roofline = the HIP events of the profiled blocks of the same window"}
    if world > 1:
        rec["ranks"] = {"elapsed_s_min": min(rank_times), "elapsed_s_max": max(rank_times),
                        "spread": max(rank_times) / min(rank_times) - 1.0, "per_rank_galaxies": N}
    if gather_ms is not None:
        rec["gather_ms"] = gather_ms
        rec["gather"] = {"bytes_per_rank_received": gathered_bytes, "ms": gather_ms,
                         "GBs_per_rank": gathered_bytes / (gather_ms * 1e-3) / 1e9,
                         "backend": backend,
                         "note": "all_gather_into_tensor of every rank's [N, 1, H, W] fp32 output into the whole "
                                 "batch on every rank (gdeconv.dist.gather_batch)"}
        rec["with_gather"] = with_gather
    if graphed is not None:
        rec["graphed"] = graphed
    if ingest is not None:
        rec["ingest"] = ingest

    if rank == 0 and world == 1 and not args.no_e2e and not rl:
        # the whole model with the ResUNet denoiser (PyTorch fp32, MIOpen, NHWC) on a sample, micro-batched
        # by the model; priced against the fp32 MFMA peak (the denoiser's convolutions dominate)
        progress("end to end with the ResUNet denoiser")
        model.Z = denoiser
        G = min(args.e2e_sample, N)
        o2, p2, a2 = obs[:G].contiguous(), psf[:G].contiguous(), alpha[:G].contiguous()
        with torch.no_grad():
            model(o2, p2, a2)
            torch.cuda.synchronize()
            te = time.perf_counter()
            for _ in range(args.e2e_forwards):
                model(o2, p2, a2)
            torch.cuda.synchronize()
            te = time.perf_counter() - te
        gal_e2e = G * args.e2e_forwards / te
        flop_gal = resunet_flops(L) * n
        rec["end_to_end"] = {"value": gal_e2e, "unit": "galaxies/s", "ms_per_forward": te * 1e3 / args.e2e_forwards,
                             "denoiser_flop_per_galaxy": flop_gal,
                             "fp32_ceiling_galaxies_s": FP32_PEAK_TFLOPS * 1e12 / flop_gal,
                             "frac_of_fp32_ceiling": gal_e2e * flop_gal / (FP32_PEAK_TFLOPS * 1e12),
                             "sample": f"{G} galaxies, full model with PyTorch ResUNet (fp32, MIOpen, NHWC), "
                                       f"{args.e2e_forwards} timed forwards after one warm forward"}
        if L <= 64 and not args.no_graph:
            # small stamps: the host's ~60 launches per forward set the eager pace; the whole model (ResUNet included)
            # replayed as one hipGraph (gdeconv.graphs.GraphedForward, the serving path of SURVEY 8(f) rank 2)
            from gdeconv.graphs import GraphedForward
            gf = GraphedForward(model, o2, p2, a2)
            gf.replay()
            torch.cuda.synchronize()
            tg = time.perf_counter()
            for _ in range(args.e2e_forwards):
                gf.replay()
            torch.cuda.synchronize()
            tg = time.perf_counter() - tg
            gal_g = G * args.e2e_forwards / tg
            rec["end_to_end"]["graphed"] = {"value": gal_g, "unit": "galaxies/s",
                                            "ms_per_forward": tg * 1e3 / args.e2e_forwards,
                                            "frac_of_fp32_ceiling": gal_g * flop_gal / (FP32_PEAK_TFLOPS * 1e12),
                                            "note": "the same sample's forward captured once (GraphedForward) and replayed"}
            del gf
        del o2, p2, a2
    if world > 1:
        dist.barrier()   # every rank's GPU work and collectives are done before rank 0 loads the host cores
    if rank == 0 and not args.no_cpu_baseline:
        progress("CPU baseline (the oracle on the host cores)")
        rec["cpu_baseline"] = cpu_baseline(args)
        if world > 1:
            rec["cpu_baseline"]["note"] = "rank 0, after every rank's timed and collective work"
    return rec


if __name__ == "__main__":
    main()
