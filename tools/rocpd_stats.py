"""Summarise a rocprofv3 rocpd database (``*_results.db``) into per-kernel stats.

usage: python tools/rocpd_stats.py gpurun_out/prof/run_results.db [out.csv] [--by-grid]

Prints the top kernels (calls, total ms, avg us, % of GPU kernel time) and writes the
full table as CSV.  ``--by-grid`` splits each kernel by launch grid, which separates
the GEMM shapes hipBLASLt picks the same kernel for.
"""
from __future__ import annotations

import csv
import sqlite3
import sys


def stats(db: str, by_grid: bool = False):
    c = sqlite3.connect(db)
    key = "name, grid_x, grid_y, grid_z, workgroup_x" if by_grid else "name"
    rows = list(c.execute(
        f"select {key}, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        f"from kernels group by {key} order by sum(duration) desc"))
    total = sum(r[-4] for r in rows) or 1
    out = []
    for r in rows:
        name = r[0] if not by_grid else f"{r[0]} grid={r[1]}x{r[2]}x{r[3]} wg={r[4]}"
        n, tot, avg, mn, mx = r[-5:]
        out.append({"Name": name, "Calls": n, "TotalDurationNs": int(tot), "AverageNs": round(avg, 1),
                    "Percentage": round(100.0 * tot / total, 3), "MinNs": int(mn), "MaxNs": int(mx)})
    return out, total


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    by_grid = "--by-grid" in sys.argv
    rows, total = stats(args[0], by_grid)
    if len(args) > 1:
        with open(args[1], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    print(f"total kernel time {total / 1e6:.1f} ms over {sum(r['Calls'] for r in rows)} dispatches")
    for r in rows[:30]:
        print(f"{r['Percentage']:6.2f}%  {r['Calls']:7d}  {r['AverageNs'] / 1e3:9.1f} us  {r['Name'][:150]}")


if __name__ == "__main__":
    main()
