"""Loop census of one kernel in a device .s: for each backward branch, the instruction
mix of the loop body (MFMA / VALU / SALU / LDS / VMEM / waitcnt / barrier).

usage: python tools/isa_loops.py /tmp/knn.s knn_filter_q256_kernelILi384E
"""
import collections
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(pat), l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith("\t.size") or ".Lfunc_end" in lines[i] and lines[i].endswith(":"))
    body = lines[start:end]
    labels = {l.split(":")[0]: k for k, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
    for k, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
        if not m:
            continue
        t = m.group(1) or m.group(2)
        if labels.get(t, 1 << 30) >= k:
            continue
        c = collections.Counter()
        for x in body[labels[t]:k + 1]:
            x = x.strip()
            if not x or x.startswith(";") or x.startswith(".") or x.endswith(":"):
                continue
            op = x.split()[0]
            if "mfma" in op:
                c["mfma"] += 1
            elif op.startswith("v_"):
                c["valu"] += 1
            elif op.startswith("s_waitcnt"):
                c["waitcnt"] += 1
            elif op.startswith("s_barrier"):
                c["barrier"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("global_", "buffer_", "flat_")):
                c["vmem"] += 1
            else:
                c[op] += 1
        print(f"loop {labels[t]}..{k} ({k - labels[t]} lines): {dict(c)}")


if __name__ == "__main__":
    main()
