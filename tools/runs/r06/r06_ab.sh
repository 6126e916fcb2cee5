#!/bin/bash
# Round 6: presleep 0 vs 1.5 vs 2 us (GCS_SERVER_PRESLEEP_NS), four rounds
# alternating, thread series 1 / 8 / 16 / 24 unpinned.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06ab}
mkdir -p $O
ss() { local name=$1; shift; env SS_PROF=0 SS_RINGS= "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json,sys; d=json.load(open('$O/$name.json'))
print('$name', {k: (v['us_per_call'], v['cpu_frac']) for k, v in d.items() if k.startswith('threads')})"; }
for r in 1 2 3 4; do
for p in 0 1500 2000; do
ss ps${p}_$r SS_THREADS=1,8,16,24 MT_PIN=0 GCS_SERVER_PRESLEEP_NS=$p
done
done
