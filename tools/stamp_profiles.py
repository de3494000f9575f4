"""Stamp one gpu_round.sh pass: does the profile of the dominant kernel reproduce the bench line's
roofline fraction, on the same box and the same kernel sources?  

    python tools/stamp_profiles.py --tag r5z --commit abc1234 --stats gpurun_out/prof_r5z/run_kernel_stats.csv \
        --pmc gpurun_out/pmc_r5z/summary.json --bench gpurun_out/bench_r5z.json --out gpurun_out/stamp_r5z.json

Writes: the dominant kernel (the bench line's roofline.kernel), its average launch time under rocprofv3
(--kernel-trace --stats, the profiled bench run) and by HIP events in the bench line (un-profiled, the same
box, the same call), the fraction of the dense peak each gives, their ratio, the effective clock of its
launches in the PMC pass (GRBM_GUI_ACTIVE / 8 / wall, MI355X_MICROARCH 'DVFS give-back'), the box's
images/s, and the kernel-source hashes of the profile, the PMC summary and the library timed.
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
from pmc_summary import label_of  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--commit", default=None)
    ap.add_argument("--stats", required=True)
    ap.add_argument("--pmc", required=True)
    ap.add_argument("--bench", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    line = json.loads(open(a.bench).read().strip().splitlines()[-1])
    roof = line["roofline"]
    dom = roof["kernel"]
    rows = {label_of(r["Name"]): r for r in csv.DictReader(open(a.stats))}
    r = rows.get(dom)
    prof_ms = float(r["AverageNs"]) / 1e6 if r else None
    gflop = roof["gflop_per_launch"]
    peak = roof["peak"]
    pmc = json.load(open(a.pmc))
    from unet_mi355x.native import kernel_sources_sha256
    out = {
        "tag": a.tag, "commit": a.commit, "kernel": dom,
        "rocprof_avg_launch_ms": round(prof_ms, 4) if prof_ms else None,
        "rocprof_calls": int(r["Calls"]) if r else None,
        "bench_event_avg_launch_ms": roof["avg_launch_ms"],
        "frac_from_rocprof": round(gflop / prof_ms / peak, 4) if prof_ms else None,
        "frac_bench_line": roof["frac"],
        "rocprof_over_events": round(prof_ms / roof["avg_launch_ms"], 4) if prof_ms else None,
        "pmc_clock_ghz": pmc.get(dom, {}).get("clock_ghz"),
        "pmc_traffic_bytes_per_launch": pmc.get(dom, {}).get("hbm_bytes_per_launch"),
        "box_images_per_s": line["value"], "box_ms_per_step": line["ms_per_step"],
        "kernel_sources_sha256_library": kernel_sources_sha256(),
        "kernel_sources_sha256_pmc": pmc.get("_meta", {}).get("kernel_sources_sha256"),
        "bench_kernel_sources_match": roof.get("kernel_sources_match"),
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
