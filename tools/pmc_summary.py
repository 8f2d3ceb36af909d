"""Merge rocprofv3 hardware-counter passes over tools/pmc_kernels.py into one per-kernel table.

Each pass is its own rocprofv3 run (`--pmc <group> --kernel-trace --output-format csv -d DIR/pN`);
this script reads every `*counter_collection.csv` under DIR, groups dispatches by
(kernel, grid, workgroup) and cuts each group into consecutive chunks of ITERS dispatches (one
chunk = one shape of pmc_kernels.py, launched ITERS times back to back), and reports the median
dispatch of each chunk.  Chunks are numbered in order of first appearance, which is the order of
the shapes in pmc_kernels.py.

    python tools/pmc_summary.py gpurun_out/pmc "title" > profiles/x.md

Derived columns (MI355X: 256 CUs x 4 SIMDs, ~2.4 GHz shader clock):
  HBM rd  = 2 x FETCH_SIZE / time   (gfx950 FETCH_SIZE counts half of a wide coalesced stream;
            MI355X_MICROARCH.md sec. HBM -- the raw value is also shown)
  wr      = WRITE_SIZE / time
  L2 hit  = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  MFMA    = SQ_VALU_MFMA_BUSY_CYCLES / (time x clock x 1024 SIMDs)
  TF      = SQ_INSTS_VALU_MFMA_MOPS_{BF16,F8} x 512 / time
  LDS cf  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait    = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

ITERS = 6
CLOCK_HZ = 2.4e9
SIMDS = 256 * 4


def _col(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    return None


def load(dirpath):
    """-> {dispatch_id: {"name", "grid", "wg", "dur_ns", counters...}} merged over passes.
    Dispatch ids restart per pass, so each pass is keyed by (pass, dispatch) and passes are
    aligned by the dispatch's position among same-(name, grid, wg) dispatches."""
    passes = []
    for path in sorted(glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)):
        disp = {}
        for r in csv.DictReader(open(path)):
            did = int(_col(r, "Dispatch_Id", "Correlation_Id"))
            d = disp.setdefault(did, {"name": _col(r, "Kernel_Name"), "grid": _col(r, "Grid_Size"),
                                      "wg": _col(r, "Workgroup_Size"), "c": {}})
            d["c"][_col(r, "Counter_Name")] = float(_col(r, "Counter_Value"))
            s, e = _col(r, "Start_Timestamp"), _col(r, "End_Timestamp")
            if s and e:
                d["dur_ns"] = int(e) - int(s)
        trace = glob.glob(os.path.join(os.path.dirname(path), "*kernel_trace.csv"))
        if trace:
            for r in csv.DictReader(open(trace[0])):
                did = int(_col(r, "Dispatch_Id", "Correlation_Id"))
                if did in disp:
                    disp[did]["dur_ns"] = int(_col(r, "End_Timestamp")) - int(_col(r, "Start_Timestamp"))
        passes.append(disp)
    return passes


def chunks(disp):
    """-> list of (first_dispatch, key, [dispatch dicts]) in order of appearance."""
    groups = defaultdict(list)
    for did in sorted(disp):
        d = disp[did]
        groups[(d["name"], d["grid"], d["wg"])].append((did, d))
    out = []
    for key, lst in groups.items():
        for i in range(0, len(lst) - ITERS + 1, ITERS):
            part = lst[i:i + ITERS]
            out.append((part[0][0], key, [d for _, d in part]))
    out.sort(key=lambda t: t[0])
    return out


def ours(name):
    return not (name.startswith("void at::") or name.startswith("at::") or name.startswith("__amd")
                or name.startswith("Cijk") or "rocclr" in name)


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def main():
    dirpath, title = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "hardware counters"
    program = sys.argv[3] if len(sys.argv) > 3 else "tools/pmc_kernels.py"
    passes = load(dirpath)
    merged = {}  # chunk index -> {"name", "dur": [...], counters: [...]}
    for disp in passes:
        idx = 0
        for _, key, lst in chunks(disp):
            if not ours(key[0]):
                continue
            m = merged.setdefault(idx, {"key": key, "dur": [], "c": defaultdict(list)})
            if m["key"] != key:  # passes disagree on the chunk sequence: keep the first pass's
                idx += 1
                continue
            for d in lst[1:]:  # first launch of a shape is cold
                if "dur_ns" in d:
                    m["dur"].append(d["dur_ns"])
                for c, v in d["c"].items():
                    m["c"][c].append(v)
            idx += 1

    def med(m, c):
        v = m["c"].get(c)
        return statistics.median(v) if v else None

    print(f"# {title}\n")
    print(f"Source: rocprofv3 `--pmc` passes under `{dirpath}` ({len(passes)} passes), program "
          f"`{program}`; median of launches 2..6 of each shape. Derivations: see "
          "`tools/pmc_summary.py` docstring (HBM rd doubles FETCH_SIZE, gfx950 counts half).\n")
    print("| # | kernel | grid | us | HBM rd GB/s (raw) | wr GB/s | L2 hit | MFMA busy | TFLOP/s | "
          "LDS confl | wave wait |")
    print("|---:|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for idx in sorted(merged):
        m = merged[idx]
        if not m["dur"]:
            continue
        t = statistics.median(m["dur"]) * 1e-9
        fs, ws = med(m, "FETCH_SIZE"), med(m, "WRITE_SIZE")
        hit, miss = med(m, "TCC_HIT_sum"), med(m, "TCC_MISS_sum")
        busy = med(m, "SQ_VALU_MFMA_BUSY_CYCLES")
        mops = (med(m, "SQ_INSTS_VALU_MFMA_MOPS_BF16") or 0) + (med(m, "SQ_INSTS_VALU_MFMA_MOPS_F8") or 0)
        bank, ldsa = med(m, "SQ_LDS_BANK_CONFLICT"), med(m, "SQ_LDS_IDX_ACTIVE")
        wait, wcyc = med(m, "SQ_WAIT_ANY"), med(m, "SQ_WAVE_CYCLES")

        def f(v, fmt):
            return "-" if v is None else fmt.format(v)

        rd = f(fs, "{:.0f}") if fs is None else f"{2 * fs * 1024 / t / 1e9:.0f} ({fs * 1024 / t / 1e9:.0f})"
        print(f"| {idx} | `{short(m['key'][0])}` | {m['key'][1]} | {t * 1e6:.1f} | {rd} | "
              f"{f(None if ws is None else ws * 1024 / t / 1e9, '{:.0f}')} | "
              f"{f(None if hit is None or hit + miss == 0 else hit / (hit + miss), '{:.2f}')} | "
              f"{f(None if busy is None else busy / (t * CLOCK_HZ * SIMDS), '{:.1%}')} | "
              f"{f(mops * 512 / t / 1e12 if mops else None, '{:.1f}')} | "
              f"{f(None if bank is None or not ldsa else bank / ldsa, '{:.1%}')} | "
              f"{f(None if wait is None or not wcyc else wait / wcyc, '{:.0%}')} |")


if __name__ == "__main__":
    main()
