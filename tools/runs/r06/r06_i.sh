#!/bin/bash
# Round 6: the varying-request stress on one ring; the C2 step's TX write-back
# as lines (default) vs nt sectors vs sc1 sectors.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread -k "every_size_and_mode or failed_wait or registered_rooms" > $O/pytest_host.log 2>&1 || { tail -40 $O/pytest_host.log; exit 1; }
tail -1 $O/pytest_host.log
for r in 1 2; do
for v in line nt sc1; do
case $v in line) E="";; nt) E="GCS_TX_LINE_WB_MB=0";; sc1) E="GCS_TX_LINE_WB_MB=0 GCS_TX_HYBRID=off";; esac
env $E timeout -k 10 180 python -u tools/step_ab.py > $O/step_${v}_$r.json 2> $O/step_${v}_$r.err || { tail -5 $O/step_${v}_$r.err; exit 1; }
python -c "
import json; d=json.load(open('$O/step_${v}_$r.json')); print('$v', d['fused_ms_median'], d['fused_event_ms_median'], d['split_ms_median'])"
done; done
