"""Phase occupancy over time from a k_gal_reg phase trace (tools/kbench_reg built with -DGD_FUSED_TRACE=1 writes
gpurun_out/kreg_trace.bin: 16 s_memrealtime stamps per workgroup, 100 MHz).  Prints, every 20 us of the launch,
how many workgroups are resident and how many are in each memory-heavy phase (z load, column A update, column B),
and the per-round mean workgroup duration: phase-locked CUs show up as all 256 in one phase at once.

usage: python tools/trace_occupancy.py gpurun_out/kreg_trace.bin
"""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16).astype(np.int64)
s = t - t[:, 0].min()
T = s[:, 9].max()
bins = np.arange(0, T, 50)  # 0.5 us


def occ(a, b):
    c = np.zeros(len(bins))
    for lo, hi in zip(s[:, a], s[:, b]):
        c[(bins >= lo) & (bins < hi)] += 1
    return c


z, ca, cb, tot = occ(0, 1), occ(3, 4), occ(6, 7), occ(0, 9)
print(f"{len(s)} workgroups, launch span {T / 100:.1f} us")
order = np.argsort(s[:, 0])
dur = (s[:, 9] - s[:, 0]) / 100
for r in range(0, len(s) // 256):
    idx = order[256 * r:256 * (r + 1)]
    print(f"round {r:2d}: starts {s[idx, 0].min() / 100:8.1f} .. {s[idx, 0].max() / 100:8.1f} us, mean duration {dur[idx].mean():6.1f} us")
print("    time   resident  z-load  col-A  col-B")
for k in range(0, len(bins), 40):
    print(f"{bins[k] / 100:8.1f}   {tot[k]:6.0f}  {z[k]:6.0f} {ca[k]:6.0f} {cb[k]:6.0f}")
