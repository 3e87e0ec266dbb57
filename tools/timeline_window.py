"""GPU busy/idle breakdown of the LAST --window-s seconds of a rocprofv3 --kernel-trace
database (rocpd SQLite): busy fraction (union of kernel intervals over all streams),
kernel time by category, and the longest idle gaps (offset into the window, length).
Point it at a bench run whose timed steps are the tail of the trace.

usage: python tools/timeline_window.py DB --window-s 7.4 [--gaps 15]
"""
import argparse
import collections
import sqlite3

# Library kernels (hipBLASLt / Tensile "Cijk_*") and hand-written kernels are kept in
# separate categories so a summary can never credit one for the other.
CATS = [("hipblaslt_MT256x256", lambda n, g: "Cijk" in n and "MT256x256" in n),
        ("hipblaslt_other", lambda n, g: "Cijk" in n or "hipblaslt" in n.lower()),
        ("gemm_pp(hand,prefill)", lambda n, g: "gemm_pp" in n or "gemm_prefill" in n),
        ("dgemm/skinny(hand,decode)", lambda n, g: "skinny" in n or "gemv" in n or "splitk" in n or "dgemm" in n),
        ("encoder_gemm", lambda n, g: "gemm_fused" in n),
        ("decode_attn", lambda n, g: "decode_attn" in n),
        ("prefill_attn", lambda n, g: "prefill_attn" in n),
        ("knn", lambda n, g: "knn" in n),
        ("norm/rope/act", lambda n, g: any(s in n for s in ("rmsnorm", "rope", "silu", "layernorm", "gelu"))),
        ("sampling", lambda n, g: "sample" in n or "logprob" in n or "topk" in n),
        ("copies", lambda n, g: "copyBuffer" in n or "copy_kernel" in n or "fillBuffer" in n),
        ("aten_other", lambda n, g: "at::native" in n),
        ("other", lambda n, g: True)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window-s", type=float, required=True)
    ap.add_argument("--gaps", type=int, default=15)
    ap.add_argument("--top", type=int, default=25, help="kernels (by name and grid) listed by time in the window")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    k = c.execute("select start, end, name, grid_x from kernels order by start").fetchall()
    t_end = max(r[1] for r in k)
    t0 = t_end - a.window_s * 1e9
    k = [r for r in k if r[1] > t0]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _, _ in k:
        s = max(s, t0)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, cur_e - t0))
            elif s > t0:
                gaps.append((s - t0, 0))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    win = t_end - t0
    print(f"window {win / 1e9:.3f} s  kernels {len(k)}  GPU busy {busy / win * 100:.1f} %  idle {(win - busy) / 1e6:.1f} ms")
    cat = collections.Counter()
    for s, e, n, g in k:
        for name, pred in CATS:
            if pred(n, g):
                cat[name] += e - max(s, t0)
                break
    tot = sum(cat.values()) or 1
    for name, v in cat.most_common():
        print(f"  {name:20s} {v / 1e6:9.1f} ms  {v / tot * 100:5.1f} % of kernel time")
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n, g in k:
        base = n[5:] if n.startswith("void ") else n
        base = base.replace("(anonymous namespace)::", "")
        key = (base.split("(")[0][-70:], g)
        per[key][0] += e - max(s, t0)
        per[key][1] += 1
    print("top kernels in the window (ms, calls, avg us, grid, name):")
    for (n, g), (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"  {t / 1e6:8.1f} {c:6d} {t / c / 1e3:8.1f} {g:9d}  {n}")
    gaps.sort(reverse=True)
    print("longest idle gaps (ms @ offset s):",
          ", ".join(f"{d / 1e6:.1f}@{o / 1e9:.2f}" for d, o in gaps[: a.gaps]))
    small = sum(d for d, _ in gaps if d < 1e6)
    print(f"idle in gaps < 1 ms: {small / 1e6:.1f} ms over {sum(1 for d, _ in gaps if d < 1e6)} gaps")


if __name__ == "__main__":
    main()
