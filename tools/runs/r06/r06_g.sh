#!/bin/bash
# Round 6: the fused step's block order (GCS_STEP_ORDER tx / rx / mix):
# parity under each order, then the C2 and C4 step A/B.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06g}
mkdir -p $O
for ord in rx mix; do
GCS_STEP_ORDER=$ord timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_step_$ord.log 2>&1 || { tail -40 $O/pytest_step_$ord.log; exit 1; }
tail -1 $O/pytest_step_$ord.log
done
for r in 1 2; do for ord in tx rx mix; do
GCS_STEP_ORDER=$ord timeout -k 10 180 python -u tools/step_ab.py > $O/step_${ord}_$r.json 2> $O/step_${ord}_$r.err || { tail -5 $O/step_${ord}_$r.err; exit 1; }
python -c "
import json; d=json.load(open('$O/step_${ord}_$r.json')); print('$ord', d['fused_ms_median'], d['fused_event_ms_median'], d['split_ms_median'])"
done; done
for ord in tx rx mix; do
SA_FRAMES=4194304 GCS_STEP_ORDER=$ord timeout -k 10 180 python -u tools/step_ab.py > $O/step4m_${ord}.json 2> $O/step4m_${ord}.err || { tail -5 $O/step4m_${ord}.err; exit 1; }
python -c "
import json; d=json.load(open('$O/step4m_${ord}.json')); print('4M $ord', d['fused_ms_median'], d['fused_event_ms_median'], d['split_ms_median'])"
done
