"""Per-decode-step summary from a rocprofv3 --kernel-trace CSV of the RAG bench.

usage: python tools/decode_step_stats.py <rocprof output dir>
Decode steps are delimited by the f32 LM-head GEMM (hipBLASLt 'BSS' kernel); prints the
median step span, decode-attention time per layer and rope_cache time per layer over
18 steps sampled across the run.
"""
import collections
import csv
import glob
import statistics
import sys


def main(d):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    with open(f) as fh:
        ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Grid_Size_X"])
                    for r in csv.DictReader(fh))
    idx = [i for i, e in enumerate(ev) if "decode_attn_kernelILi128ELi1" in e[2]]
    spans = []
    for frac in [x / 20 for x in range(2, 20)]:
        j = idx[int(len(idx) * frac)]
        while "BSS" not in ev[j][2]:
            j -= 1
        k = j + 1
        while "BSS" not in ev[k][2]:
            k += 1
        agg = collections.defaultdict(lambda: [0, 0.0])
        for s, e, n, g in ev[j + 1: k + 1]:
            key = n[:120] + " g" + g
            agg[key][0] += 1
            agg[key][1] += (e - s) / 1e3
        at = [v for kk, v in agg.items() if "decode_attn" in kk][0]
        rope = sum(v[1] for kk, v in agg.items() if "rope_cache" in kk)
        spans.append(((ev[k][1] - ev[j][1]) / 1e3, at[1] / at[0], rope / 32))
    med = [statistics.median(x[i] for x in spans) for i in range(3)]
    print("median decode step %.1f us, decode attention %.1f us/layer, rope_cache %.1f us/layer" % tuple(med))


if __name__ == "__main__":
    main(sys.argv[1])
