#!/bin/bash
# Round 6: a sleep right after posting (GCS_SERVER_PRESLEEP_NS, A/B knob) before
# the spin: thread series 1 / 8 / 16 / 24 unpinned (the box's quota: 16 CPUs),
# presleep 0 / 2 / 3 / 4 us, two rounds alternating; 8 / 16 pinned at 0 and 3 us.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06aa}
mkdir -p $O
ss() { local name=$1; shift; env SS_PROF=0 SS_RINGS= "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json,sys; d=json.load(open('$O/$name.json'))
print('$name', {k: (v['us_per_call'], v['cpu_frac']) for k, v in d.items() if k.startswith('threads')})"; }
for r in 1 2; do
for p in 0 2000 3000 4000; do
ss ps${p}_$r SS_THREADS=1,8,16,24 MT_PIN=0 GCS_SERVER_PRESLEEP_NS=$p
done
done
ss pin_ps0 SS_THREADS=8,16 MT_PIN=1 GCS_SERVER_PRESLEEP_NS=0
ss pin_ps3000 SS_THREADS=8,16 MT_PIN=1 GCS_SERVER_PRESLEEP_NS=3000
