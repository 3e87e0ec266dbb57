"""Host/GPU hand-off analysis of a rocprofv3 (--kernel-trace --hip-trace) database:
for every decode graph step, when the host called hipGraphLaunch relative to the end of
the previous GPU work on the same stream, and how long the call took.  Prints a small
summary (the database itself can be too big to copy back).

usage: python tools/gap_analysis.py DB [--window-s 5]
"""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window-s", type=float, default=5.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    views = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    print("views:", [v for v in views if not v.startswith("rocpd_") or v in ("rocpd_region",)][:20])
    api_view = next((v for v in ("regions", "rocpd_region") if v in views), None)
    cols = [r[1] for r in c.execute(f"pragma table_info({api_view})")] if api_view else []
    print("api view", api_view, cols[:20])
    k = c.execute("select start, end, name from kernels where stream_id=0 order by start").fetchall()
    t_end = max(r[1] for r in k)
    t0 = t_end - a.window_s * 1e9
    launches = []
    if api_view:
        launches = c.execute(f"select start, end from {api_view} where name like '%GraphLaunch%' and start > ? "
                             "order by start", (t0,)).fetchall()
    print("graph launches in window:", len(launches))
    gi = [i for i in range(1, len(k)) if "gather_feedback" in k[i][2] and k[i][0] > t0]
    import bisect
    ls = [x[0] for x in launches]
    rel_start, dur, gap, first_after = [], [], [], []
    for i in gi:
        prev_end = max(r[1] for r in k[max(0, i - 3): i])
        j = bisect.bisect_right(ls, k[i][0]) - 1   # the last launch call before the step's first kernel
        if j < 0:
            continue
        s, e = launches[j]
        rel_start.append((s - prev_end) / 1e3)    # host call start relative to previous GPU work end
        dur.append((e - s) / 1e3)
        gap.append((k[i][0] - prev_end) / 1e3)
        first_after.append((k[i][0] - e) / 1e3)   # first kernel after the call returned
    if gap:
        q = lambda v: (round(statistics.median(v), 1), round(sorted(v)[len(v) // 10], 1), round(sorted(v)[9 * len(v) // 10], 1))
        print("steps", len(gap))
        print("GPU gap before step (median, p10, p90 us):", q(gap))
        print("hipGraphLaunch call start - previous GPU end (us):", q(rel_start))
        print("hipGraphLaunch duration (us):", q(dur))
        print("first kernel - call end (us):", q(first_after))


if __name__ == "__main__":
    main()
