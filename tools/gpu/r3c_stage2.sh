# RAG bench with stage + search tracers
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LS_STAGE_TRACE=1 timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/stage2_r3c.log 2>&1
rc=$?; grep '"metric"' gpurun_out/stage2_r3c.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_s'], d['step_phases_rank0_s'])
for st in d.get('stage_trace_rank0_s', []):
    se = st.pop('searches', [])
    print(st); print('  searches', se)"; exit $rc
