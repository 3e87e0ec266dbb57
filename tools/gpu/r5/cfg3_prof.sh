# r5: config 3 under rocprofv3 --kernel-trace: kernel mix of the timed window (the last
# 3 steps) vs the whole run (setup included: random-init weights, cache fills).
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r5s}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/prof_cfg3_$T -o pc -- python3 bench.py --config chat --steps 3 --warmup 1 > gpurun_out/cfg3_prof_$T.log 2>&1 || { tail -30 gpurun_out/cfg3_prof_$T.log; exit 1; }
grep '"metric"' gpurun_out/cfg3_prof_$T.log | cut -c1-300
DB=$(find gpurun_out/prof_cfg3_$T -name '*.db' | head -1)
python3 tools/rocpd_stats.py $DB --top 25 > gpurun_out/cfg3_stats_all_$T.txt
python3 tools/timeline_window.py $DB --window-s 2.1 --top 30 > gpurun_out/cfg3_timeline_$T.txt
head -40 gpurun_out/cfg3_timeline_$T.txt | cut -c1-200
rm -f $DB
