#!/bin/bash
# Round 6: k_desc_stream without flat stores (the RX verdict and the per-frame
# path's outputs straight to global memory, no LDS sink): the GPU suite on the
# new build, then the bench's C3 and rooms tables A/B, alternating the two
# libraries (mtcp_amd/lib_ab/{old,new}.so).
set -o pipefail
O=gpurun_out/${R06_OUT:-r06y}
LIB=mtcp_amd/lib/libmtcp_gpucsum.so
mkdir -p $O
cp mtcp_amd/lib_ab/new.so $LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_new.log 2>&1 || { tail -40 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
for r in 1 2; do for v in old new; do
cp mtcp_amd/lib_ab/$v.so $LIB
timeout -k 10 420 python -u bench.py --cpu-seconds 0 > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -20 $O/bench_${v}_$r.err; exit 1; }
cp profiles/bench_extras_last.json $O/bench_extras_${v}_$r.json
python -c "
import json; d=json.load(open('$O/bench_extras_${v}_$r.json')); c=d['c2_rooms']; i=d['c3_imix']
print('$v $r', d['value'], {k: round(c[k]*1e3,1) for k in ('stream_verify_ms','stream_compute_ms','rooms_verify_ms')}, {k: round(i[k]*1e3,1) for k in ('verify_ms','compute_ms','compute_ms_cold','verify_ms_cold')})"
done; done
cp mtcp_amd/lib_ab/new.so $LIB
