"""Summarise rocprofv3 PMC passes into per-kernel HBM traffic per launch.

usage: python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv>
                                   <out.json> --batch N --size L

Counters come from two separate passes (`rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`; the
TCC slots cannot hold both).  Per MI355X_MICROARCH.md (HBM section) on gfx950 FETCH_SIZE reports
exactly half the bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane streaming stores.  Both are in KiB.  Values are per launch, averaged over the
launches of each kernel, and summed over the counter's instances (XCDs).
"""
import argparse
import collections
import csv
import json
import re

MODE_NAMES = {
    "k_row_fwd": ["ITER", "PSF_Y", "PSF_YP", "PSF_RAW", "PSF", "ONE", "TWO", "YA"],
    "k_col": ["ITER", "OTF_INIT", "OTF_CONV", "WIENER", "OTF", "CONV", "CONVC", "CONV2", "FWD", "INV",
              "G_INIT", "G_ITER", "G_W1", "G_ITER_F", "G_ITER_L", "G_ITER_FL"],
    "k_row_inv": ["ITER", "INIT", "OUT1", "OUT2", "RL_FINAL"],
    "k_row_invfwd": ["CLAMP", "RL_RATIO", "RL_UPDATE"],
    "k_subnet_features": ["FEATURES"],
    "k_gal_iter": ["MID", "FIRST", "LAST", "FIRST_LAST"],
}


def pretty(kname):
    if "k_subnet_features_psf" in kname:
        return "k_subnet_features<128,PSF>"       # |FFT2(pad128(psf))|^2 in the kernel, then the conv stack
    if "k_subnet_features" in kname:
        return "k_subnet_features<128,FEATURES>"
    if "k_subnet_mlp" in kname:
        return "k_subnet_mlp<128,MLP>"            # the SubNet's MLP, batched
    m = re.search(r"k_gal_small_init<(\d+)>", kname)
    if m:
        return f"k_gal_small_init<{m.group(1)}>"
    m = re.search(r"k_subnet_rhos_init<(\d+)>", kname)
    if m:
        return f"k_subnet_rhos_init<{m.group(1)}>"   # SubNet + the small-image init in one launch
    m = re.search(r"k_gal_mid_init<(\d+),", kname)
    if m:
        return f"k_gal_mid_init<{m.group(1)}>"        # fused init at the mid sizes (80 / 112 / 144 / 160)
    m = re.search(r"k_gal_(small_t|small_p|mid)<(\d+), \d+, \d+(?:, \d+)?, (true|false), (true|false)>", kname)
    if m:  # the transposing-plan iterations: k_gal_small's role names (48^2), k_gal_mid's own (80..160^2)
        first, last = m.group(3) == "true", m.group(4) == "true"
        base = "k_gal_mid" if m.group(1) == "mid" else "k_gal_small"
        return f"{base}<{m.group(2)},{['MID', 'FIRST', 'LAST', 'FIRST_LAST'][first + 2 * last]}>"
    m = re.search(r"k_gal_small<(\d+), (true|false), (true|false)>", kname)
    if m:
        first, last = m.group(2) == "true", m.group(3) == "true"
        return f"k_gal_small<{m.group(1)},{['MID', 'FIRST', 'LAST', 'FIRST_LAST'][first + 2 * last]}>"
    m = re.search(r"k_gal_reg_init<(\d+)(?:, (true|false))?>", kname)
    if m:
        return f"k_gal_init<{m.group(1)},{'POIS' if m.group(2) == 'true' else 'REG'}>"  # fused init (512 threads)
    m = re.search(r"k_pois_b<(\d+)>", kname)
    if m:
        return f"k_pois_b<{m.group(1)}>"              # Poisson pass B
    m = re.search(r"k_rl_reg<(\d+)>", kname)
    if m:
        return f"k_rl_reg<{m.group(1)}>"              # whole Richardson-Lucy loop per galaxy
    m = re.search(r"k_gal_reg<(\d+)(?:, (true|false))?>", kname)
    if m:
        if m.group(2) == "true":
            return f"k_pois_a<{m.group(1)}>"          # Poisson pass A
        return f"k_gal_reg<{m.group(1)}>"             # fused iteration (first / middle / last: runtime flags)
    m = re.search(r"(k_gal_iter2?)<(\d+), (true|false), (true|false)(?:, (\d+))?>", kname)
    if m:
        if m.group(5) == "1":
            return f"k_gal_init<{m.group(2)},Y>"      # fused init: y -> |H|^2, G, zin
        if m.group(5) == "3":
            return f"k_gal_init<{m.group(2)},ONE>"    # fused init in one launch: y -> |H|^2, G, zin, W~
        first, last = m.group(3) == "true", m.group(4) == "true"
        return f"{m.group(1)}<{m.group(2)},{['MID', 'FIRST', 'LAST', 'FIRST_LAST'][first + 2 * last]}>"
    m = re.search(r"k_gal_w1<(\d+)>", kname)
    if m:
        return f"k_gal_init<{m.group(1)},W1>"         # fused init: zin -> W~
    m = re.search(r"k_psf_rows<(\d+)(, (true|false))?>", kname)
    if m:
        return f"k_psf_rows<{m.group(1)},{'STATE' if m.group(3) == 'true' else 'ROWS'}>"
    m = re.search(r"(k_\w+)<(\d+), (\d+)(?:, \d+)?>", kname)
    if not m:
        return None
    k, L, mode = m.group(1), m.group(2), int(m.group(3))
    return f"{k}<{L},{MODE_NAMES[k][mode]}>"


def per_launch(path, counter):
    sums = collections.defaultdict(float)   # (kernel, dispatch) -> value
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = pretty(r.get("Kernel_Name", ""))
        if name:
            sums[(name, r.get("Dispatch_Id"))] += float(r["Counter_Value"])
    by_k = collections.defaultdict(list)
    for (name, _), v in sums.items():
        by_k[name].append(v)
    return {k: sum(v) / len(v) for k, v in by_k.items()}, {k: len(v) for k, v in by_k.items()}


def dispatch_order(path, counter):
    """[(dispatch id, kernel, value)] of one counter pass in dispatch order (every profiled engine kernel)."""
    sums = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = pretty(r.get("Kernel_Name", ""))
        if name:
            sums[(int(r.get("Dispatch_Id")), name)] += float(r["Counter_Value"])
    return [(d, k, v) for (d, k), v in sorted(sums.items())]


def init_pass_b(path, counter, L):
    """Mean per launch of the Poisson init's own pass B (k_pois_b<INIT>: the k_pois_b dispatch that follows a
    k_gal_reg_init<POIS> dispatch) and of the iterations' pass B, from one counter pass; None when absent."""
    seq = dispatch_order(path, counter)
    ini, it = [], []
    for i, (_, k, v) in enumerate(seq):
        if k != f"k_pois_b<{L}>":
            continue
        (ini if i > 0 and seq[i - 1][1] == f"k_gal_init<{L},POIS>" else it).append(v)
    if not ini:
        return None
    return sum(ini) / len(ini), (sum(it) / len(it) if it else 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--iters", type=int, default=None,
                    help="ADMM iterations in the profiled run (default: the init kernel's launches x --n-iters; "
                         "bench --steps 1 --warmup 1 runs 3 forwards: warmup, timed region, profiling pass)")
    ap.add_argument("--rl-calls", type=int, default=0,
                    help="Richardson-Lucy workload (any value > 0 selects it): forwards in the profiled run, "
                         "overridden by the k_rl_reg launch count when that kernel ran; "
                         "op_richardson_lucy<L> = every engine kernel's bytes / calls")
    ap.add_argument("--n-iters", type=int, default=None, help="iterations per forward of the profiled workload")
    a = ap.parse_args()
    fetch, nf = per_launch(a.fetch, "FETCH_SIZE")
    write, _ = per_launch(a.write, "WRITE_SIZE")
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "galaxy-deconv_amd"))
    from gdeconv import _lib
    out = {"batch": a.batch, "size": a.size, "engine_rev": _lib.load().gd_engine_rev().decode(),
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; FETCH_SIZE x2 (gfx950 "
                     "half-counting of wide streaming reads, MI355X_MICROARCH.md HBM section); KiB -> bytes",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        rd = 2 * fetch.get(k, 0.0) * 1024
        wr = write.get(k, 0.0) * 1024
        out["kernels"][k] = {"read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                             "hbm_bytes_per_launch": rd + wr, "launches": nf.get(k, 0)}
    # whole Gaussian ADMM iteration (RF(z) -> C_G_ITER[0] -> RI(zin), all chunks): traffic per call
    L = a.size
    if a.iters is None:  # forwards in the run = launches of the one-per-forward init kernel
        fw = 0
        for k in (f"k_gal_init<{L},REG>", f"k_gal_init<{L},POIS>", f"k_gal_small_init<{L}>", f"k_gal_mid_init<{L}>",
                  f"k_subnet_rhos_init<{L}>", f"k_gal_init<{L},ONE>", f"k_gal_init<{L},W1>"):
            fw = fw or out["kernels"].get(k, {}).get("launches", 0)
        a.iters = fw * (a.n_iters or 8) if fw else 24
    if a.rl_calls and f"k_rl_reg<{L}>" in out["kernels"]:
        a.rl_calls = out["kernels"][f"k_rl_reg<{L}>"]["launches"]
    members = [f"k_row_fwd<{L},ONE>", f"k_col<{L},G_ITER>", f"k_col<{L},G_ITER_F>", f"k_col<{L},G_ITER_L>",
               f"k_row_inv<{L},OUT1>", f"k_gal_iter<{L},MID>", f"k_gal_iter<{L},FIRST>", f"k_gal_iter<{L},LAST>",
               f"k_gal_reg<{L}>", f"k_gal_small<{L},MID>", f"k_gal_small<{L},FIRST>", f"k_gal_small<{L},LAST>",
               f"k_gal_small<{L},FIRST_LAST>", f"k_gal_mid<{L},MID>", f"k_gal_mid<{L},FIRST>", f"k_gal_mid<{L},LAST>",
               f"k_gal_mid<{L},FIRST_LAST>"]
    tot = sum(v["hbm_bytes_per_launch"] * v["launches"] for k, v in out["kernels"].items() if k in members)
    if tot:
        out["kernels"][f"op_admm_iter<{L},Gaussian>"] = {
            "hbm_bytes_per_launch": tot / a.iters, "launches": a.iters,
            "note": "sum over the iteration's RF/C/RI chunk launches; FETCH/WRITE_SIZE count L2<->fabric "
                    "traffic, Infinity-Cache hits included"}
    pois = [f"k_pois_a<{L}>", f"k_pois_b<{L}>"]
    if any(k in out["kernels"] for k in pois):  # Poisson two-pass: pass A (every iteration) + pass B (not the last)
        ptot = sum(v["hbm_bytes_per_launch"] * v["launches"] for k, v in out["kernels"].items() if k in pois)
        nb = out["kernels"].get(f"k_pois_b<{L}>", {}).get("launches", 0)
        na = out["kernels"].get(f"k_pois_a<{L}>", {}).get("launches", 0)
        # pass B's launches include the init's one per forward; a.iters = iterations in the run
        init_b = max(0, nb - (na - na // max(1, a.n_iters or 8)))
        out["kernels"][f"op_admm_iter<{L},Poisson>"] = {
            "hbm_bytes_per_launch": (ptot - init_b * out["kernels"][f"k_pois_b<{L}>"]["hbm_bytes_per_launch"]) / a.iters,
            "launches": a.iters, "note": "Poisson two-pass: pass A + pass B per call (the init's pass B excluded)"}
    if f"k_gal_init<{L},POIS>" in out["kernels"] and f"k_pois_b<{L}>" in out["kernels"]:
        pi = [f"k_psf_rows<{L},STATE>", f"k_gal_init<{L},POIS>"]
        # the init's pass B (k_pois_b<INIT>: no w read) apart from the iterations' (w read): round 5 priced the init
        # with the average over both, i.e. (n - 1) / n of an image too many (the 1.10x "excess" of
        # profiles/r05i_pmc_summary_poisson.txt was that accounting)
        fb, wb = init_pass_b(a.fetch, "FETCH_SIZE", L), init_pass_b(a.write, "WRITE_SIZE", L)
        if fb and wb:
            pb_init, pb_iter = 2 * fb[0] * 1024 + wb[0] * 1024, 2 * fb[1] * 1024 + wb[1] * 1024
            ni = out["kernels"][f"k_gal_init<{L},POIS>"]["launches"]
            nb = out["kernels"][f"k_pois_b<{L}>"]["launches"]
            out["kernels"][f"k_pois_b<{L},INIT>"] = {"hbm_bytes_per_launch": pb_init, "launches": ni}
            out["kernels"][f"k_pois_b<{L},ITER>"] = {"hbm_bytes_per_launch": pb_iter, "launches": nb - ni}
            pa = out["kernels"].get(f"k_pois_a<{L}>")
            if pa and f"op_admm_iter<{L},Poisson>" in out["kernels"]:
                it = out["kernels"][f"op_admm_iter<{L},Poisson>"]["launches"]
                out["kernels"][f"op_admm_iter<{L},Poisson>"]["hbm_bytes_per_launch"] = \
                    (pa["hbm_bytes_per_launch"] * pa["launches"] + pb_iter * (nb - ni)) / it
                out["kernels"][f"op_admm_iter<{L},Poisson>"]["note"] = \
                    "Poisson two-pass: pass A + the iterations' pass B per call (the init's pass B apart)"
            note = "k_psf_rows<STATE> + k_gal_reg_init<POIS> + the init's own pass B (k_pois_b<INIT>)"
        else:
            pb_init = out["kernels"][f"k_pois_b<{L}>"]["hbm_bytes_per_launch"]
            note = "k_psf_rows<STATE> + k_gal_reg_init<POIS> + one pass B (its per-launch average)"
        out["kernels"][f"op_admm_init<{L},Poisson>"] = {
            "hbm_bytes_per_launch": sum(out["kernels"][k]["hbm_bytes_per_launch"] for k in pi if k in out["kernels"])
            + pb_init,
            "launches": out["kernels"][f"k_gal_init<{L},POIS>"]["launches"], "note": "Poisson init: " + note}
    init = [f"k_psf_rows<{L},STATE>", f"k_gal_init<{L},Y>", f"k_gal_init<{L},W1>"]
    if f"k_gal_init<{L},ONE>" in out["kernels"]:
        init = [f"k_psf_rows<{L},STATE>", f"k_gal_init<{L},ONE>"]
    if f"k_gal_init<{L},REG>" in out["kernels"]:
        init = [f"k_psf_rows<{L},STATE>", f"k_gal_init<{L},REG>"]
    if f"k_gal_small_init<{L}>" in out["kernels"]:
        init = [f"k_gal_small_init<{L}>"]
    if f"k_gal_mid_init<{L}>" in out["kernels"]:
        init = [f"k_gal_mid_init<{L}>"]
    if all(k in out["kernels"] for k in init):
        out["kernels"][f"op_admm_init<{L},Gaussian>"] = {
            "hbm_bytes_per_launch": sum(out["kernels"][k]["hbm_bytes_per_launch"] for k in init),
            "launches": out["kernels"][init[-1]]["launches"],
            "note": "fused init: " + " + ".join(init) + ", per call"}
    if f"k_subnet_rhos_init<{L}>" in out["kernels"]:
        v = out["kernels"][f"k_subnet_rhos_init<{L}>"]
        out["kernels"][f"op_admm_init_subnet<{L},Gaussian>"] = {
            "hbm_bytes_per_launch": v["hbm_bytes_per_launch"], "launches": v["launches"],
            "note": "SubNet + fused small-image init in one launch (k_subnet_rhos_init), per call"}
    if a.rl_calls:
        tot = sum(v["hbm_bytes_per_launch"] * v["launches"] for v in out["kernels"].values())
        out["kernels"][f"op_richardson_lucy<{L}>"] = {
            "hbm_bytes_per_launch": tot / a.rl_calls, "launches": a.rl_calls,
            "note": "every engine kernel of the Richardson-Lucy forward, per call"}
    if a.n_iters is not None:
        out["n_iters"] = a.n_iters
    json.dump(out, open(a.out, "w"), indent=1)
    for k, v in out["kernels"].items():
        if "read_bytes_per_launch" in v:
            print(f"{k:28s} read {v['read_bytes_per_launch'] / 1e9:8.3f} GB  write "
                  f"{v['write_bytes_per_launch'] / 1e9:8.3f} GB  x{v['launches']}")
        else:
            print(f"{k:28s} total {v['hbm_bytes_per_launch'] / 1e9:8.3f} GB per call  x{v['launches']}")


if __name__ == "__main__":
    main()
