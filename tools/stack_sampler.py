"""Whole-process Python stack sampler: run a script in-process and sample every thread's
stack every few ms (cProfile only sees the thread it runs in).  Prints the hottest leaf
lines and inclusive functions.

usage: python tools/stack_sampler.py [--every-ms 2] [--top 40] [--thread PREFIX] -- script.py args...

--thread PREFIX: only threads whose name starts with PREFIX, leaves keyed by their last
three frames (where that thread spends its wall time, waits included).
"""
import collections
import os
import runpy
import sys
import threading
import time
import traceback


def main():
    argv = sys.argv[1:]
    every, top = 0.002, 40
    only = None
    while argv and argv[0] != "--":
        if argv[0] == "--thread":
            only = argv[1]
            argv = argv[2:]
            continue
        if argv[0] == "--every-ms":
            every = float(argv[1]) / 1000.0
            argv = argv[2:]
        elif argv[0] == "--top":
            top = int(argv[1])
            argv = argv[2:]
        else:
            raise SystemExit(__doc__)
    argv = argv[1:]
    sys.path.insert(0, os.path.dirname(os.path.abspath(argv[0])))
    leaf, incl = collections.Counter(), collections.Counter()
    busy = collections.Counter()
    stop = threading.Event()

    def sampler():
        me = threading.get_ident()
        names = {}
        while not stop.is_set():
            for t in threading.enumerate():
                names[t.ident] = t.name
            for tid, fr in sys._current_frames().items():
                if tid == me:
                    continue
                if only is not None and not names.get(tid, "").startswith(only):
                    continue
                st = traceback.extract_stack(fr)
                if not st:
                    continue
                f = st[-1]
                key = f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}"
                if only is not None:
                    key = " < ".join(f"{os.path.basename(g.filename)}:{g.lineno}:{g.name}" for g in st[-3:][::-1])
                leaf[key] += 1
                # a thread parked in a wait / socket read / select is idle
                if not any(s in key for s in ("wait", "_recv_exact", "select", "sleep", "get", "accept")):
                    busy[names.get(tid, str(tid)).split("-")[0]] += 1
                seen = set()
                for g in st:
                    k = f"{os.path.basename(g.filename)}:{g.name}"
                    if k not in seen:
                        incl[k] += 1
                        seen.add(k)
            time.sleep(every)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    sys.argv = argv
    try:
        runpy.run_path(argv[0], run_name="__main__")
    except SystemExit:
        pass
    finally:
        stop.set()
        th.join(1)
        print("== busy samples by thread", file=sys.stderr)
        for k, n in busy.most_common(15):
            print(f"{n:8d} {k}", file=sys.stderr)
        print("== leaf lines", file=sys.stderr)
        for k, n in leaf.most_common(top):
            print(f"{n:8d} {k}", file=sys.stderr)
        print("== inclusive", file=sys.stderr)
        for k, n in incl.most_common(top * 2):
            print(f"{n:8d} {k}", file=sys.stderr)


if __name__ == "__main__":
    main()
