#!/bin/bash
# Round 6: what the uncached-frames acquire (buffer_inv sc0) costs: the RX split
# with the default acquire vs GCS_SERVER_ACQUIRE=none (no acquire at all; A/B
# only), counting grid and plain, alternating.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06p}
mkdir -p $O
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/rx_split.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.load(open('$O/$name.json')); print('$name', {k: d[k] for k in ('call_us_median','post_to_done_us','gpu_span_us','acquire_us','frames_us','records_us','wrong_verdicts')})"; }
for r in 1 2; do
run rxs_inv_$r
run rxs_none_$r GCS_SERVER_ACQUIRE=none
run rxs_inv_plain_$r GCS_SERVER_COUNTERS=0
run rxs_none_plain_$r GCS_SERVER_COUNTERS=0 GCS_SERVER_ACQUIRE=none
done
