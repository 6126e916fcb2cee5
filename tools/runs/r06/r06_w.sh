#!/bin/bash
# Round 6: the burst server with no flat memory ops left (request-line polls
# and the frames' 2 B stores through the global address space) against the
# build before: the server/plugin GPU tests on the new build, then the RX
# split A/B, alternating the two libraries (mtcp_amd/lib_ab/{old,new}.so).
set -o pipefail
O=gpurun_out/${R06_OUT:-r06w}
LIB=mtcp_amd/lib/libmtcp_gpucsum.so
mkdir -p $O
cp mtcp_amd/lib_ab/new.so $LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_new.log 2>&1 || { tail -40 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/rx_split.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.load(open('$O/$name.json')); print('$name', {k: d[k] for k in ('call_us_median','post_to_done_us','poll_us','seen_poll_us','gpu_span_us','acquire_us','frames_us','wrong_verdicts')})"; }
for r in 1 2 3; do
for v in old new; do
cp mtcp_amd/lib_ab/$v.so $LIB
run rxs_${v}_$r
run rxs_${v}_plain_$r GCS_SERVER_COUNTERS=0
done
done
cp mtcp_amd/lib_ab/new.so $LIB
