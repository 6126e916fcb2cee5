#!/bin/bash
# Round 6: frame loads through the global address space (global_load) vs the
# flat loads the burst server compiled to before: the server/plugin/step GPU
# tests on the new build, then the RX split A/B, alternating the two libraries
# (mtcp_amd/lib_ab/{flat,global}.so, built in the container) in place.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06o}
LIB=mtcp_amd/lib/libmtcp_gpucsum.so
mkdir -p $O
cp mtcp_amd/lib_ab/global.so $LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_global.log 2>&1 || { tail -40 $O/pytest_global.log; exit 1; }
tail -1 $O/pytest_global.log
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/rx_split.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.load(open('$O/$name.json')); print('$name', {k: d[k] for k in ('call_us_median','post_to_done_us','gpu_span_us','acquire_us','frames_us','records_us','wrong_verdicts')})"; }
for r in 1 2; do
for v in flat global; do
cp mtcp_amd/lib_ab/$v.so $LIB
run rxs_${v}_$r
run rxs_${v}_plain_$r GCS_SERVER_COUNTERS=0
run rxs_pg_${v}_plain_$r GCS_SERVER_COUNTERS=0 RXS_ROOMS=pageable
done
done
cp mtcp_amd/lib_ab/global.so $LIB
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'])"
