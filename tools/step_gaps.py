"""Per-decode-step GPU timeline from a rocprofv3 database: where the GPU idles between kernels.

    python tools/step_gaps.py gpurun_out/prof_head/run_results.db

A decode step is delimited by the sampler kernel (sample_partial / sample_final).  For the steps
of the timed region it reports the median GPU-busy time, the median idle gap between consecutive
kernels inside a step, and the median idle gap from one step's last kernel to the next step's
first kernel (the host's token -> next launch critical path)."""
import sqlite3
import statistics
import sys


def main():
    path = sys.argv[1]
    c = sqlite3.connect(path)
    ks = c.execute("select name, start, end from kernels order by start").fetchall()
    steps, cur = [], []
    for name, s, e in ks:
        cur.append((name, s, e))
        if "sample_final" in name or ("sample" in name and "partial" not in name):
            steps.append(cur)
            cur = []
    # keep decode steps: those with a chain_kernel launch
    dec = [st for st in steps if any("chain_kernel" in n for n, _, _ in st)]
    dec = dec[len(dec) // 3:]  # skip warm-up
    busy, inner, between, lead = [], [], [], {}
    for st in dec:
        busy.append(sum(e - s for _, s, e in st) / 1e3)
        for (n0, s0, e0), (n1, s1, e1) in zip(st, st[1:]):
            g = (s1 - e0) / 1e3
            inner.append(g)
            key = f"{n0[:40]} -> {n1[:40]}"
            lead.setdefault(key, []).append(g)
    for a, b in zip(dec, dec[1:]):
        between.append((b[0][1] - a[-1][2]) / 1e3)
    print(f"decode steps analysed: {len(dec)}")
    print(f"median GPU busy per step: {statistics.median(busy):.1f} us")
    print(f"median wall per step (first start -> last end): "
          f"{statistics.median([(st[-1][2] - st[0][1]) / 1e3 for st in dec]):.1f} us")
    print(f"median sum of inner gaps per step: "
          f"{statistics.median([sum((b[1] - a[2]) / 1e3 for a, b in zip(st, st[1:])) for st in dec]):.1f} us")
    print(f"median step-to-step gap (last kernel end -> next step first kernel): "
          f"{statistics.median(between):.1f} us (p10 {sorted(between)[len(between) // 10]:.1f})")
    print("largest median inner gaps:")
    for k, v in sorted(lead.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1]))[:12]:
        print(f"  {statistics.median(v):8.1f} us x{len(v):5d}  {k}")


if __name__ == "__main__":
    main()
