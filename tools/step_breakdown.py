"""Per-step kernel time of a tools/r02_fullstep.sh trace (rocprofv3 SQLite output): the
steps after the first five, split at the optimizer kernel.
usage: python tools/step_breakdown.py <run_results.db> [top]"""
import collections
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
opt = [i for i, r in enumerate(rows) if "sgd" in r[0] or "adam" in r[0]]
sub = rows[opt[4] + 1: opt[-1] + 1]
n = len(opt) - 5
span = (sub[-1][2] - sub[0][1]) / 1e3 / n
busy = sum(e - s for _, s, e in sub) / 1e3 / n
print(f"steps {n}  {span:.1f} us/step wall  {busy:.1f} us/step kernel-busy  "
      f"{len(sub) // n} launches/step")
agg = collections.defaultdict(lambda: [0, 0])
for name, s, e in sub:
    agg[name][0] += 1
    agg[name][1] += e - s
for name, (k, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{t / 1e3 / n:8.1f} us/step {k // n:3d}x {t / k / 1e3:7.1f} us  {name[:96]}")
