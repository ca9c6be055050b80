"""Static instruction counts of the engine's kernels (device ISA): VALU / packed VALU / LDS / VMEM / SALU / branch
per kernel, plus VGPRs and spills, for A/B-ing instruction-count changes on the CPU before a GPU run.

    python tools/isa_count.py [--filter k_rl_reg] [-D NAME=VALUE ...]

Compiles csrc/gd_engine.hip with the library's flags (device code only, -S) into /tmp and walks each kernel's body.
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))


def classify(op):
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith(("v_mfma", "v_smfmac")):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--filter", default="")
    p.add_argument("-D", action="append", default=[])
    p.add_argument("--out", default="/tmp/gd_isa.s")
    args = p.parse_args()
    from gdeconv import _lib
    flags = [f for f in _lib.BUILD_FLAGS if f not in ("-shared", "-fPIC")]
    cmd = ["/opt/rocm/bin/hipcc", *flags, "--cuda-device-only", "-S", *[f"-D{d}" for d in args.D], "-o", args.out,
           os.path.join(ROOT, "galaxy-deconv_amd", "csrc", "gd_engine.hip")]
    subprocess.run(cmd, check=True, cwd=os.path.join(ROOT, "galaxy-deconv_amd", "csrc"))
    kern, counts, meta, rows = None, None, {}, []
    for line in open(args.out):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            kern, counts = m.group(1), {}
            rows.append((kern, counts))
            continue
        m = re.match(r"^\s*\.(vgpr_count|vgpr_spill_count|agpr_count|sgpr_spill_count):\s*(\d+)", line)
        if m:
            continue
        m = re.search(r";\s*(NumVgprs|ScratchSize|NumAgprs):\s*(\d+)", line)
        if m and kern:
            meta.setdefault(kern, {})[m.group(1)] = int(m.group(2))
            continue
        if kern is None:
            continue
        if line.startswith("\t.end_amdgpu") or line.startswith(".Lfunc_end"):
            kern = None
            continue
        s = line.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c = classify(op)
        counts[c] = counts.get(c, 0) + 1
    names = subprocess.run(["c++filt"], input="\n".join(k for k, _ in rows), capture_output=True,
                           text=True).stdout.split("\n")
    cols = ["valu", "valu_pk", "lds", "vmem", "salu", "wait", "barrier", "branch", "mfma"]
    print(f"{'kernel':64s} " + " ".join(f"{c:>7s}" for c in cols) + f" {'vgpr':>5s} {'scr':>5s}")
    for (k, c), n in zip(rows, names):
        n = n.replace("void gd::", "").replace("(gd::Args)", "").replace("(gd::Args, int)", "")
        if args.filter not in n:
            continue
        m = meta.get(k, {})
        print(f"{n[:64]:64s} " + " ".join(f"{c.get(x, 0):7d}" for x in cols)
              + f" {m.get('NumVgprs', -1):5d} {m.get('ScratchSize', -1):5d}")


if __name__ == "__main__":
    main()
