"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_pmc.sh).

Usage: python scripts/pmc_summary.py <root> <workload> [calibration json]
<root>_FETCH_SIZE/ and <root>_WRITE_SIZE/ hold one pass each.  Per kernel: the
average per launch over the launches of 1M datagrams (the counters are KiB).

Calibration (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only for known
access shapes): the ceiling kernel in 'read only' mode reads exactly 12 B
(offset + length) + 64 B (head) per datagram and writes 1 B, so
fetch_scale = expected_read_bytes / FETCH_SIZE for that shape; the parse
kernels' reads have the same shape and get the same scale (a workload without
the ceiling run takes the scale of the calibration json).
"""
import collections
import csv
import glob
import json
import sys

root, workload = sys.argv[1], sys.argv[2]
KEYS = (("ceil_kernel<1>", "ceil_read_only"), ("ceil_kernel<0>", "ceil_rw"), ("ceil_kernel<2>", "ceil_write_only"),
        ("ceil_kernel<3>", "ceil_rw_lds"), ("rtps_parse_spec_kernel", "parse_spec"),
        ("rtps_parse_chain_kernel", "parse_chain"), ("rtps_parse_lds_kernel", "parse_lds"),
        ("rtps_parse_fix_kernel", "parse_fix"), ("rtps_parse_item_kernel", "parse_item"),
        ("rtps_parse_emit_kernel", "parse_emit"), ("rtps_parse_emit2_kernel", "parse_emit2"), ("rtps_parse_scan_kernel", "parse_scan"),
        ("rtps_parse_rslab_kernel", "parse_rslab"), ("rtps_parse_rcopy_kernel", "parse_rcopy"))
vals = collections.defaultdict(lambda: collections.defaultdict(list))
grid = collections.defaultdict(list)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{root}_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            key = next((k for pat, k in KEYS if pat in name), None)
            if key is None:
                continue
            # only the launches over the whole 1M-datagram batch (4096 tiles of 256 for the parse)
            g = int(r.get("Grid_Size", r.get("Grid_Size_X", "0")) or 0)
            grid[key].append(g)
            vals[key][c].append((g, float(r["Counter_Value"]) * 1024.0))
n = 1 << 20
out = {"source": f"{root}_{{FETCH_SIZE,WRITE_SIZE}} (scripts/gpu_pmc.sh)", "datagrams_per_launch": n,
       "workload": workload}
for k, d in vals.items():
    big = max(g for g, _ in d.get("FETCH_SIZE", d.get("WRITE_SIZE", [(0, 0)])))
    out[k] = {c: sum(v for g, v in lst if g == big) / max(1, sum(1 for g, _ in lst if g == big))
              for c, lst in d.items()}
    out[k]["grid"] = big
fs = out.get("ceil_read_only", {}).get("FETCH_SIZE")
if fs:
    out["fetch_scale"] = n * (12 + 64) / fs
elif len(sys.argv) > 3:
    out["fetch_scale"] = json.load(open(sys.argv[3])).get("fetch_scale")
    out["fetch_scale_source"] = sys.argv[3]
print(json.dumps(out, indent=1))
