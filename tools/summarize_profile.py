"""rocprofv3 --stats output -> markdown table for profiles/ (top kernels by total time).

    python tools/summarize_profile.py gpurun_out/prof2/run_kernel_stats.csv "title" > profiles/x.md
    python tools/summarize_profile.py gpurun_out/prof_head/run_results.db "title" > profiles/x.md

Accepts the CSV kernel-stats file or the rocpd SQLite database (`run_results.db`, the default
output format of rocprofv3 in ROCm 7.x); from the database it also lists each top kernel's
register / LDS / scratch footprint.
"""
import csv
import sqlite3
import sys


def _rows_csv(path):
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
             float(r["Percentage"]), None) for r in csv.DictReader(open(path))]


def _rows_db(path):
    c = sqlite3.connect(path)
    res = c.execute("select name, count(*), sum(duration), max(vgpr_count), max(accum_vgpr_count), "
                    "max(sgpr_count), max(lds_size), max(scratch_size) from kernels group by name "
                    "order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in res) or 1.0
    return [(r[0], r[1], float(r[2]), float(r[2]) / r[1], 100.0 * r[2] / tot,
             f"{r[3]}/{r[4]}/{r[5]}/{r[6]}/{r[7]}") for r in res]


def main():
    path, title = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "kernel stats"
    rows = _rows_db(path) if path.endswith(".db") else _rows_csv(path)
    tot = sum(r[2] for r in rows)
    res = rows[0][5] is not None if rows else False
    print(f"# {title}\n")
    print(f"Source: `{path}` (rocprofv3 --kernel-trace --stats). Total GPU kernel time {tot / 1e6:.1f} ms.\n")
    print("| kernel | calls | total ms | avg us | % |" + (" vgpr/agpr/sgpr/lds/scratch |" if res else ""))
    print("|---|---:|---:|---:|---:|" + ("---|" if res else ""))
    for name, calls, total, avg, pct, footprint in rows[:30]:
        name = name.replace("|", "/").replace("(anonymous namespace)::", "")
        if len(name) > 110:
            name = name[:110] + "..."
        print(f"| `{name}` | {calls} | {total / 1e6:.2f} | {avg / 1e3:.2f} | {pct:.2f} |"
              + (f" {footprint} |" if res else ""))


if __name__ == "__main__":
    main()
