"""Per-dispatch PMC counters of a rocprofv3 --pmc run, in dispatch order, with the kernel label.

    python tools/pmc_dispatches.py gpurun_out/pmc_dir [--grep ring8] [--min-ms 0.1]

Prints dispatch id, duration (ms, from the pass's kernel trace), kernel label (tools/pmc_summary.label_of)
and every counter; FETCH_SIZE is also shown as HBM-side read GB with the gfx950 x2 correction
(MI355X_MICROARCH.md §HBM), WRITE_SIZE as GB.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_clock import load  # noqa: E402
from pmc_summary import label_of  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--grep", default="")
    ap.add_argument("--min-ms", type=float, default=0.0)
    a = ap.parse_args()
    rows = load(a.dir)
    for did in sorted(rows):
        r = rows[did]
        lab = label_of(r.get("name", "?"))
        ms = r.get("ms", 0.0)
        if a.grep not in lab or ms < a.min_ms:
            continue
        c = r["ctr"]
        extra = ""
        if "FETCH_SIZE" in c:
            extra += f" read {2 * c['FETCH_SIZE'] * 1024 / 1e9:7.3f} GB"
        if "WRITE_SIZE" in c:
            extra += f" write {c['WRITE_SIZE'] * 1024 / 1e9:7.3f} GB"
        print(f"{did:6d} {ms:8.3f} ms{extra}  {lab}")


if __name__ == "__main__":
    main()
