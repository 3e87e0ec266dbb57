"""Per-kernel time summary from a rocprofv3 SQLite database (rocpd format).

usage: python tools/rocpd_stats.py gpurun_out/prof/x_results.db [--grid] [--top 30]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--grid", action="store_true", help="split rows by grid size")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    key = "name, grid_x" if a.grid else "name"
    rows = c.execute(f"select {key}, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     f"from kernels group by {key} order by sum(duration) desc").fetchall()
    total = sum(r[-4] for r in rows) or 1
    print("pct,total_us,calls,avg_us,min_us,max_us," + ("grid," if a.grid else "") + "name")
    for r in rows[: a.top]:
        name = r[0]
        short = (name if name.startswith("(") or name.startswith("void (") else name.split("(")[0])[:110]
        g = f"{r[1]}," if a.grid else ""
        n, s, avg, mn, mx = r[-5:]
        print(f"{100 * s / total:.2f},{s / 1e3:.1f},{n},{avg / 1e3:.2f},{mn / 1e3:.2f},{mx / 1e3:.2f},{g}{short}")


if __name__ == "__main__":
    main()
