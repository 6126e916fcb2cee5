#!/bin/bash
# Round 6: the server's block shape (GCS_SERVER_SHAPE 32x3 / 64x2): parity of
# the server tests under 64x2, then the RX split and thread series both ways.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06m}
mkdir -p $O
GCS_SERVER_SHAPE=64x2 timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_plugin.py tests/test_plugin_faults.py tests/test_gpu_mt.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_64x2.log 2>&1 || { tail -40 $O/pytest_64x2.log; exit 1; }
tail -1 $O/pytest_64x2.log
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/rx_split.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.load(open('$O/$name.json')); print('$name', {k: d[k] for k in ('call_us_median','post_to_done_us','gpu_span_us','acquire_us','frames_us','records_us','wrong_verdicts')})"; }
for r in 1 2; do
run rxs_32x3_$r
run rxs_64x2_$r GCS_SERVER_SHAPE=64x2
run rxs_32x3_plain_$r GCS_SERVER_COUNTERS=0
run rxs_64x2_plain_$r GCS_SERVER_COUNTERS=0 GCS_SERVER_SHAPE=64x2
run rxs_pg_32x3_plain_$r GCS_SERVER_COUNTERS=0 RXS_ROOMS=pageable
run rxs_pg_64x2_plain_$r GCS_SERVER_COUNTERS=0 RXS_ROOMS=pageable GCS_SERVER_SHAPE=64x2
done
ss() { local name=$1; shift; env SS_PROF=0 SS_RINGS=4x4 "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json,sys; d=json.load(open('$O/$name.json'))
print('$name', {k: (v.get('us_per_call', v.get('us_per_round')), v['cpu_frac']) for k, v in d.items() if k.startswith('threads') or k.startswith('rings')})"; }
ss ss_32x3 SS_THREADS=1,8,16 MT_PIN=1
ss ss_64x2 SS_THREADS=1,8,16 MT_PIN=1 GCS_SERVER_SHAPE=64x2
