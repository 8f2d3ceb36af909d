"""Per-kernel duration and launch gap (previous kernel's end -> this kernel's start) from a
rocprofv3 kernel trace database, for back-to-back (graph) launch sequences.

    python tools/trace_gaps.py gpurun_out/x/run_results.db "title" [--max-gap-us 20] > profiles/x.md

Only gaps below --max-gap-us count (a larger one is the host between graph replays)."""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("title")
    ap.add_argument("--max-gap-us", type=float, default=20.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    try:
        rows = c.execute("select name, start, end from kernels order by start").fetchall()
    except sqlite3.Error:
        cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
        raise SystemExit(f"kernels columns: {cols}")
    per = {}
    gaps_all = []
    for i, (name, s, e) in enumerate(rows):
        d = per.setdefault(name, {"dur": [], "gap": []})
        d["dur"].append((e - s) / 1e3)
        if i:
            g = (s - rows[i - 1][2]) / 1e3
            if 0 <= g < a.max_gap_us:
                d["gap"].append(g)
                gaps_all.append(g)
    print(f"# {a.title}\n")
    print(f"Source: `{a.db}`; {len(rows)} kernels; launch gaps < {a.max_gap_us} us: {len(gaps_all)}, "
          f"median {statistics.median(gaps_all) if gaps_all else 0:.2f} us, "
          f"mean {statistics.mean(gaps_all) if gaps_all else 0:.2f} us\n")
    print("| kernel | calls | total ms | median us | mean us | median gap before us |")
    print("|---|---:|---:|---:|---:|---:|")
    items = sorted(per.items(), key=lambda kv: -sum(kv[1]["dur"]))
    for name, d in items[:30]:
        n = name.replace("|", "/").replace("(anonymous namespace)::", "")
        if len(n) > 110:
            n = n[:107] + "..."
        gap = f"{statistics.median(d['gap']):.2f}" if d["gap"] else "-"
        print(f"| `{n}` | {len(d['dur'])} | {sum(d['dur']) / 1e3:.2f} | {statistics.median(d['dur']):.2f} | "
              f"{statistics.mean(d['dur']):.2f} | {gap} |")


if __name__ == "__main__":
    main()
