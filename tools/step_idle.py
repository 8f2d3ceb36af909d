"""GPU idle time per LLM decode step from a rocprofv3 kernel trace of the headline bench: the
union of kernel intervals is subtracted from the span between consecutive step launches (the
chained layer kernel marks a step), so whatever the GPU spends waiting for the host -- token
readback, grammar accept, next step's metadata + graph replay -- shows up as idle.

    python tools/step_idle.py gpurun_out/x/run_results.db "title" [--step-kernel chain_kernel] > profiles/x.md

Steps whose idle exceeds --cap-us (default 2000: a new request's admission, ASR, prefill) are
counted separately and left out of the percentiles.
"""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("title")
    ap.add_argument("--step-kernel", default="chain_kernel")
    ap.add_argument("--cap-us", type=float, default=2000.0)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name, start, end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if a.step_kernel in r[0]]
    idle, busy, skipped = [], [], 0
    for i0, i1 in zip(starts, starts[1:]):
        t0, t1 = rows[i0][1], rows[i1][1]
        covered, cur_s, cur_e = 0, None, None
        for _, s, e in rows[i0:i1]:
            s, e = max(s, t0), min(e, t1)
            if e <= s:
                continue
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    covered += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            covered += cur_e - cur_s
        gap_us = (t1 - t0 - covered) / 1e3
        if gap_us > a.cap_us:
            skipped += 1
            continue
        idle.append(gap_us)
        busy.append(covered / 1e3)
    print(f"# {a.title}\n")
    print(f"Source: `{a.db}` (rocprofv3 --kernel-trace).  A step = one `{a.step_kernel}` launch to the next; "
          f"idle = step span minus the union of kernel intervals.\n")
    if not idle:
        print("no steps found")
        return
    q = statistics.quantiles(idle, n=10) if len(idle) >= 10 else [min(idle)] * 9
    print("| steps | GPU busy us (median) | idle us p10 | median | p90 | mean | steps over cap |")
    print("|---:|---:|---:|---:|---:|---:|---:|")
    print(f"| {len(idle)} | {statistics.median(busy):.1f} | {q[0]:.1f} | {statistics.median(idle):.1f} | "
          f"{q[8]:.1f} | {statistics.mean(idle):.1f} | {skipped} |")


if __name__ == "__main__":
    main()
