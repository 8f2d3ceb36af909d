"""rocprofv3 --stats CSV -> markdown table for profiles/ (top kernels by total time).

    python tools/summarize_profile.py gpurun_out/prof2/run_kernel_stats.csv "title" > profiles/x.md
"""
import csv
import sys


def main():
    path, title = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "kernel stats"
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print(f"Source: `{path}` (rocprofv3 --kernel-trace --stats). Total GPU kernel time {tot / 1e6:.1f} ms.\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for r in rows[:30]:
        name = r["Name"].replace("|", "/")
        if len(name) > 95:
            name = name[:95] + "..."
        print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
              f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main()
