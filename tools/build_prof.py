"""Kernel-time breakdown of the last wide-tree device build in a rocprofv3 --kernel-trace database
(the launches from the last sahInitKernel / plocInitKernel up to the next render kernel).

    python tools/build_prof.py gpurun_out/<dir>
"""
import glob
import sqlite3
import sys
from collections import defaultdict

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
rows = list(sqlite3.connect(db).execute("select name, start, end from kernels order by start"))
first = max(i for i, r in enumerate(rows) if "sahInitKernel" in r[0] or "plocInitKernel" in r[0])
# the build starts with the LBVH: back up to the previous render / rng kernel
while first > 0 and "render" not in rows[first - 1][0] and "rngInit" not in rows[first - 1][0]:
    first -= 1
last = first
while last < len(rows) and "renderKernel" not in rows[last][0]:
    last += 1
span = (rows[last - 1][2] - rows[first][1]) / 1e6
busy = sum(r[2] - r[1] for r in rows[first:last]) / 1e6
agg = defaultdict(lambda: [0, 0.0])
for r in rows[first:last]:
    k = r[0].replace("(anonymous namespace)::", "").replace("pt::", "").replace("void ", "").split("(")[0]
    agg[k][0] += 1
    agg[k][1] += (r[2] - r[1]) / 1e6
print(f"build span {span:.3f} ms, kernel time {busy:.3f} ms, {last - first} launches")
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {t:8.3f} ms  {n:4d}x  {k}")
