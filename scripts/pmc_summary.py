"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of scripts/diag_ceiling.py.

Calibration (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only for known
access shapes): the ceiling kernel in 'read only' mode reads exactly
12 B (offset+length) + 64 B (head) per datagram and writes 1 B, so
fetch_scale = expected_read_bytes / FETCH_SIZE_bytes for that shape.  The
parse kernel's reads have the same shape (T) and get the same scale.
Usage: python scripts/pmc_summary.py gpurun_out/pmc_ceil > profiles/<round>_pmc_T.json
"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{root}_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            key = ("ceil_read_only" if "ceil_kernel<1>" in name else "ceil_rw" if "ceil_kernel<0>" in name else
                   "ceil_write_only" if "ceil_kernel<2>" in name else "ceil_rw_lds" if "ceil_kernel<3>" in name else
                   "parse_spec" if "rtps_parse_spec_kernel" in name else "parse_fix" if "rtps_parse_fix" in name else
                   None)
            if key:
                vals[key][c].append(float(r["Counter_Value"]) * 1024.0)  # counters are KiB
n = 1 << 20
out = {"source": root, "datagrams_per_launch": n, "workload": "T (1M x 1024 B, first launches of diag_ceiling.py)"}
for k, d in vals.items():
    out[k] = {c: sum(v) / len(v) for c, v in d.items()}
exp_read = n * (12 + 64)
fs = out.get("ceil_read_only", {}).get("FETCH_SIZE")
out["fetch_scale"] = exp_read / fs if fs else None
if fs and "parse_spec" in out:
    ps = out["parse_spec"]
    out["parse_traffic_bytes"] = ps["FETCH_SIZE"] * out["fetch_scale"] + ps.get("WRITE_SIZE", 0)
    if "parse_fix" in out:
        pf = out["parse_fix"]
        out["parse_traffic_bytes"] += pf["FETCH_SIZE"] * out["fetch_scale"] + pf.get("WRITE_SIZE", 0)
print(json.dumps(out, indent=1))
