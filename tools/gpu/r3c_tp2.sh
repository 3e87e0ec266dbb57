# two-rank native TP on one GPU (gloo) + bench with prompt arrival phases
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_engine_gpu.py -k "tp2_two_ranks or tp_path_world1" -x -v --timeout 200 --timeout-method thread > gpurun_out/tp2_tests.log 2>&1
rc=$?; tail -15 gpurun_out/tp2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_phases.log 2>&1 || exit $?
grep '"metric"' gpurun_out/bench_phases.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['step_phases_rank0_s'])"
