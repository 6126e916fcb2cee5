#!/bin/bash
# Round 6: the 4M step in bench.py's timing (per-step events) vs step_ab's
# (events at the ends, alternating blocks), same box, alternating.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06r}
mkdir -p $O
for r in 1 2; do
timeout -k 10 240 python -u bench.py --no-extras --cpu-seconds 0 --frames-per-gpu 4194304 > $O/bench4m_$r.json 2> $O/bench4m_$r.err || { tail -5 $O/bench4m_$r.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench4m_$r.json')); print('bench 4M', d['value'], d['ms_per_step'], d['kernels_ms'])"
SA_FRAMES=4194304 timeout -k 10 180 python -u tools/step_ab.py > $O/step4m_$r.json 2> $O/step4m_$r.err || { tail -5 $O/step4m_$r.err; exit 1; }
python -c "
import json; d=json.load(open('$O/step4m_$r.json')); print('step_ab 4M', d['fused_ms_median'], d['fused_event_ms_median'], d['split_ms_median'])"
done
