"""Print one step's kernel sequence from a rocprofv3 --kernel-trace database: the
launches from the last kernel matching FIRST through the next matching LAST, with
each one's duration and the gap before it (us).
usage: trace_step.py DB FIRST LAST"""
import re
import sqlite3
import sys

db, first, last = sys.argv[1:4]
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end from kernels order by start"))
starts = [i for i, r in enumerate(rows) if re.search(first, r[0])]
assert starts, f"no kernel matches {first}"
i0 = starts[-2] if len(starts) > 1 else starts[-1]  # the second-to-last step: a complete one
out, prev = [], None
for name, s, e in rows[i0:]:
    short = re.sub(r"\(.*", "", name.replace("void ", "").replace("(anonymous namespace)::", ""))[-70:]
    out.append((short, (e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0))
    prev = e
    if re.search(last, name) and len(out) > 1:
        break
tot = (prev - rows[i0][1]) / 1e3
busy = sum(d for _, d, _ in out)
for n, d, g in out:
    print(f"{d:9.1f} {g:6.1f}  {n}")
print(f"step {tot:.1f} us: kernels {busy:.1f}, gaps {tot - busy:.1f}, {len(out)} launches")
