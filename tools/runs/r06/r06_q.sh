#!/bin/bash
# Round 6: the C4 step (4M + 4M) as sub-steps (GCS_STEP_SUB_FRAMES, A/B knob):
# parity of the step tests with small sub-steps, then the 4M step whole vs
# sub-steps of 1M and 2M frames, alternating.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06q}
mkdir -p $O
GCS_STEP_SUB_FRAMES=1000 timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_step_sub.log 2>&1 || { tail -40 $O/pytest_step_sub.log; exit 1; }
tail -1 $O/pytest_step_sub.log
for r in 1 2; do for sub in 0 1048576 2097152; do
SA_FRAMES=4194304 GCS_STEP_SUB_FRAMES=$sub timeout -k 10 180 python -u tools/step_ab.py > $O/step4m_${sub}_$r.json 2> $O/step4m_${sub}_$r.err || { tail -5 $O/step4m_${sub}_$r.err; exit 1; }
python -c "
import json; d=json.load(open('$O/step4m_${sub}_$r.json')); print('4M sub=$sub', d['fused_ms_median'], d['fused_event_ms_median'], d['split_ms_median'])"
done; done
