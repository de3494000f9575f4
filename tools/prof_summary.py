"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid size): calls and average ms.

    python tools/prof_summary.py gpurun_out/prof_1/run_kernel_trace.csv [--min-grid N]

The bench process also runs small warm-up / bias-centring forwards; grouping by grid size
separates the full-batch dispatches (the ones bench.py's roofline times) from those.
"""
import argparse
import os
import sys
import csv
import re
from collections import defaultdict


def short(name):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pmc_summary import label_of
    if name.startswith("_ZN4unet"):
        return label_of(name)
    m = re.search(r"igemm_kernelI(\w+?)Li(\d)ELi(\d)ELi(\d)ELi(\d)ELi(\d)E", name)
    if m:
        return f"igemm<{m.group(1)},{','.join(m.group(i) for i in range(2, 7))}>"
    m = re.search(r"igemm_kernel<[^>]*?(\d), (\d), (\d+), (\d), (\d)>", name)
    if m:
        return "igemm<?," + ",".join(m.groups()) + ">"
    return name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-grid", type=int, default=0)
    a = ap.parse_args()
    agg = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(a.trace)):
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        if g < a.min_grid:
            continue
        k = (short(r["Kernel_Name"]), g)
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':40s} {'grid':>12s} {'calls':>6s} {'avg_ms':>9s} {'total_ms':>9s} {'%':>6s}")
    for (k, g), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:40s} {g:12d} {c:6d} {t / c:9.4f} {t:9.2f} {100 * t / tot:6.2f}")


if __name__ == "__main__":
    main()
