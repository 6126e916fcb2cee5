#!/bin/bash
# Round 6: fused TX+RX step (tests, A/B), C4 pure-nt sectors, RX split with
# regions registered uncached vs cached, alternating in one box.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_step.log 2>&1 || { tail -40 $O/pytest_step.log; exit 1; }
tail -2 $O/pytest_step.log
for r in 1 2; do timeout -k 10 180 python -u tools/step_ab.py > $O/step_ab_$r.json 2> $O/step_ab_$r.err || { tail -5 $O/step_ab_$r.err; exit 1; }; cat $O/step_ab_$r.json; done
SA_FRAMES=4194304 timeout -k 10 180 python -u tools/step_ab.py > $O/step_ab_4m.json 2> $O/step_ab_4m.err || { tail -5 $O/step_ab_4m.err; exit 1; }; cat $O/step_ab_4m.json
c4() { local name=$1; shift; env "$@" timeout -k 10 180 python -u -c "
import json, torch, bench
from mtcp_amd import gpucsum
ctx = gpucsum.Context(0)
torch.cuda.set_stream(torch.cuda.Stream())
r = bench.c4_shard(ctx, torch, 20, 3, 1.0)
ctx.close()
print(json.dumps(r))" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
python -c "
import json; d=json.load(open('$O/$name.json'))
print('$name', round(d['ms_per_step'],4), 'fill', round(d['compute_ms'],4), round(d['compute_frac'],4), 'verify', round(d['verify_ms'],4), round(d['verify_frac'],4))"; }
for r in 1 2; do
c4 c4_base_$r
c4 c4_nt_$r GCS_TX_HYBRID=nt
c4 c4_ntonly_$r GCS_TX_HYBRID=nt GCS_TX_LINE_WB_MB=0
done
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/rx_split.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.load(open('$O/$name.json')); print('$name', d['call_us_median'], d['call_us_p90'], d['post_to_done_us'], d['wrong_verdicts'])"; }
for r in 1 2 3; do
run rxs_uc_$r GCS_SERVER_COUNTERS=0
run rxs_cached_$r GCS_SERVER_COUNTERS=0 GCS_REGISTER_UNCACHED=0
done
