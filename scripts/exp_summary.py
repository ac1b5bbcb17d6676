"""Summarise gpu_exp_ingest.sh outputs: per variant and workload, the ingest step and the
ingest kernels' average launch times (rocprofv3 kernel stats).

usage: python3 scripts/exp_summary.py "product v1 v2" "C3 T" [kernel-substring ...]
"""
import csv
import json
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")


def main():
    variants = sys.argv[1].split()
    wls = sys.argv[2].split()
    pats = sys.argv[3:] or ["k_"]
    for wl in wls:
        for v in variants:
            js = os.path.join(OUT, f"exp_{v}_{wl}.json")
            ks = os.path.join(OUT, f"exp_prof_{v}_{wl}", "run_kernel_stats.csv")
            if not os.path.exists(js):
                print(f"{wl:3s} {v:12s} (missing)")
                continue
            line = json.loads(open(js).read().strip().splitlines()[-1])
            ing = line.get("ingest", {}).get("ms")
            parts = []
            if os.path.exists(ks):
                for r in csv.DictReader(open(ks)):
                    name = r["Name"]
                    if any(p in name for p in pats):
                        short = name.split("::")[1].split("(")[0] if "::" in name else name[:20]
                        parts.append(f"{short} {float(r['AverageNs']) / 1e3:.1f}")
            print(f"{wl:3s} {v:12s} ingest {ing * 1e3 if ing else float('nan'):7.1f} us | " + ", ".join(parts))


if __name__ == "__main__":
    main()
