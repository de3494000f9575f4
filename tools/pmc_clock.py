"""Per-dispatch clock / MFMA utilisation / wait breakdown from rocprofv3 --pmc passes.

    python tools/pmc_clock.py gpurun_out/pmc2_def [--min-ms 0.5]

effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time (MI355X_MICROARCH.md DVFS note);
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs).
"""
import argparse
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import label_of  # noqa: E402


def load(d):
    rows = defaultdict(lambda: {"ctr": {}})
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r["Dispatch_Id"])
            rows[did]["name"] = r["Kernel_Name"]
            c = rows[did]["ctr"]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r["Dispatch_Id"])
            if did in rows:
                rows[did]["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-ms", type=float, default=0.5)
    a = ap.parse_args()
    passes = sorted(p for p in glob.glob(os.path.join(a.dir, "pass*")) if os.path.isdir(p))
    per = [load(p) for p in passes]
    # align dispatches of the last forward across passes by order
    def last_forward(r):   # the dispatches after the last forward's first launch (input pre-cast / first conv)
        d = [v for k, v in sorted(r.items()) if "unet" in v.get("name", "")]
        starts = [i for i, v in enumerate(d) if "x_to_px4" in v["name"] or "first_conv" in v["name"]]
        d = d[starts[-1] + 1:] if starts else d
        return [v for v in d if v.get("ms", 0) >= a.min_ms]
    seqs = [last_forward(r) for r in per]
    print(f"{'#':>3s} {'kernel':44s} {'ms':>7s} {'GHz':>5s} {'mfma%':>6s} {'wait%':>6s} {'winst%':>6s} {'act%':>6s} "
          f"{'L2hit%':>6s} {'ldsconf%':>8s}")
    for i in range(len(seqs[0])):
        c = {}
        for s in seqs:
            if i < len(s):
                c.update(s[i]["ctr"])
        d = seqs[0][i]
        gui = c.get("GRBM_GUI_ACTIVE", 0)
        ghz = gui / 8 / (d["ms"] * 1e-3) / 1e9 if d.get("ms") else 0
        mf = 100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui / 8 * 1024) if gui else 0
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        hit = c.get("TCC_HIT_sum", 0)
        miss = c.get("TCC_MISS_sum", 0)
        print(f"{i:3d} {label_of(d['name'])[:44]:44s} {d['ms']:7.3f} {ghz:5.2f} {mf:6.1f} "
              f"{100 * c.get('SQ_WAIT_ANY', 0) / wc:6.1f} {100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} "
              f"{100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1f} {100 * hit / max(1, hit + miss):6.1f} "
              f"{100 * c.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, c.get('SQ_LDS_IDX_ACTIVE', 0)):8.2f}")


if __name__ == "__main__":
    main()
