"""Median GPU busy / wall time per decode step, by launch form (chained + attention, chained 5..16 rows, per-kernel),
from rocprofv3 databases: python tools/step_classes.py a.db [b.db ...]"""
import sqlite3, statistics, sys
def steps(path):
    c = sqlite3.connect(path)
    ks = c.execute("select name, start, end from kernels order by start").fetchall()
    out, cur = [], []
    for n, s, e in ks:
        cur.append((n, s, e))
        if "sample_final" in n:
            out.append(cur); cur = []
    return out
for path in sys.argv[1:]:
    st = steps(path)
    cls = {}
    for s in st:
        names = " ".join(n for n, _, _ in s)
        if "chain_kernel" not in names and "skinny_stream_kernel<2, 2" not in names:
            continue
        if "true>" in names and "chain_kernel" in names: k = "chain_xg (5-16 rows)"
        elif "chain_kernel<8, 0, 4, 4" in names: k = "chain+attn (<=4 rows)"
        elif "chain_kernel" in names: k = "chain no attn"
        else: k = "per-kernel"
        busy = sum(e - b for _, b, e in s) / 1e3
        wall = (s[-1][2] - s[0][1]) / 1e3
        cls.setdefault(k, []).append((busy, wall))
    print(path)
    for k, v in sorted(cls.items()):
        print(f"  {k:24s} n={len(v):4d} busy med {statistics.median(x for x, _ in v):8.1f} us  wall med {statistics.median(y for _, y in v):8.1f} us")
