"""Deterministic profile of EVERY thread of a script (cProfile is per-thread): wraps
threading.Thread.run so each thread profiles itself, merges all threads' stats at
exit and prints the top functions by own time and by cumulative time.

usage: python tools/thread_cprofile.py [--top 50] [--cpu] -- script.py args...

--cpu times with each thread's CPU clock (time.thread_time) instead of wall time, so a
thread waiting for the GIL or a lock is not charged for it.
"""
import cProfile
import os
import pstats
import runpy
import sys
import threading

_profiles = []
_lock = threading.Lock()


def main():
    argv = sys.argv[1:]
    top = 50
    if argv[:1] == ["--top"]:
        top, argv = int(argv[1]), argv[2:]
    timer = []
    if argv[:1] == ["--cpu"]:
        import time
        timer, argv = [time.thread_time], argv[1:]
    if argv[:1] == ["--"]:
        argv = argv[1:]
    orig_run = threading.Thread.run

    def run(self):
        pr = cProfile.Profile(*timer)
        with _lock:
            _profiles.append(pr)
        pr.enable()
        try:
            orig_run(self)
        finally:
            pr.disable()

    threading.Thread.run = run
    main_pr = cProfile.Profile(*timer)
    _profiles.append(main_pr)
    sys.argv = argv
    sys.path.insert(0, os.path.dirname(os.path.abspath(argv[0])))
    main_pr.enable()
    try:
        runpy.run_path(argv[0], run_name="__main__")
    except SystemExit:
        pass
    finally:
        main_pr.disable()
        for p in _profiles:
            p.disable()
        st = None
        for p in _profiles:
            try:
                st = pstats.Stats(p) if st is None else (st.add(p) or st)
            except TypeError:   # a thread that never ran
                pass
        st.stream = sys.stderr
        st.sort_stats("tottime").print_stats(top)
        st.sort_stats("cumulative").print_stats(top)


if __name__ == "__main__":
    main()
