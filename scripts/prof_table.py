"""Print a rocprofv3 --stats kernel_stats.csv as a readable table (kernel short name, calls, avg/min/max us)."""
import csv
import re
import sys


def short(name):
    n = re.sub(r"\(.*", "", name)          # drop the argument list
    n = re.sub(r"<.*>", "<..>", n)          # collapse template arguments
    return n.split("::")[-1].strip() or name[:60]


for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    print(f"# {path}")
    print(f"{'kernel':46s} {'calls':>6s} {'avg us':>9s} {'min us':>9s} {'max us':>9s} {'total %':>8s}")
    for r in rows:
        print(f"{short(r['Name'])[:46]:46s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:9.1f} "
              f"{float(r['MinNs']) / 1e3:9.1f} {float(r['MaxNs']) / 1e3:9.1f} {float(r['Percentage']):8.2f}")
