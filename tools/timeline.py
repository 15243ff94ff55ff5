"""Per-dispatch timeline of a rocprofv3 --kernel-trace CSV: for the last N steps of a bench run, each
kernel's start offset / duration within its step and the idle gaps between consecutive kernels.
usage: python tools/timeline.py <kernel_trace.csv> [--first KERNEL_SUBSTR] [--steps 5]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--first", default="conv1_fwd_x3")
ap.add_argument("--steps", type=int, default=5)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]]
sel = starts[-a.steps - 1:]
for s0, s1 in zip(sel[:-1], sel[1:]):
    t0 = int(rows[s0]["Start_Timestamp"])
    prev_end = None
    gaps = 0.0
    for r in rows[s0:s1]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (st - prev_end) / 1e3 if prev_end is not None else 0.0
        gaps += max(gap, 0.0)
        print(f"{(st - t0) / 1e3:8.1f} us  {(en - st) / 1e3:7.1f} us  gap {gap:6.1f}  {r['Kernel_Name'].split('(')[0][:70]}")
        prev_end = en
    print(f"step {(int(rows[s1]['Start_Timestamp']) - t0) / 1e3:.1f} us, gaps {gaps:.1f} us\n")
