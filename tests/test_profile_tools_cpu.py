"""CPU checks of the trace-analysis tools that produce profiles/ summaries, on synthetic rocprofv3
kernel tables (a `kernels(name, start, end)` table in ns, like run_results.db)."""
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _db(path, rows):
    c = sqlite3.connect(path)
    c.execute("create table kernels(name text, start integer, end integer)")
    c.executemany("insert into kernels values(?, ?, ?)", rows)
    c.commit()
    c.close()


def _run(*args):
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "step_idle.py"), *args],
                          capture_output=True, text=True, check=True).stdout


def test_step_idle_counts_gaps_between_kernels_not_overlaps(tmp_path):
    """12 steps of chain (3 ms) -> LM head (40 us, overlapping the chain's tail by 10 us) -> 5 us
    gap -> sampler (5 us) -> 40 us host gap: 45 us idle per step; one step with a 5 ms admission
    gap is counted over the cap, not in the percentiles."""
    rows, t = [], 0
    for s in range(12):
        rows += [("void chain_kernel<8>(ChainParams const*)", t, t + 3_000_000),
                 ("lm_head", t + 2_990_000, t + 3_040_000),
                 ("sample_partial_kernel", t + 3_045_000, t + 3_050_000)]
        t += 3_050_000 + (5_000_000 if s == 6 else 40_000)
    db = str(tmp_path / "run_results.db")
    _db(db, rows)
    out = _run(db, "t")
    line = [l for l in out.splitlines() if l.startswith("| 10 |")]
    assert line, out
    cells = [c.strip() for c in line[0].strip("|").split("|")]
    assert float(cells[1]) == 3045.0  # busy: the union of the chain and the overlapping head
    assert float(cells[3]) == 45.0  # median idle
    assert cells[6] == "1"  # the admission step


def test_step_idle_without_steps(tmp_path):
    db = str(tmp_path / "run_results.db")
    _db(db, [("lm_head", 0, 10)])
    assert "no steps found" in _run(db, "t")
