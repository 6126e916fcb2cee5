#!/bin/bash
# Round 6: yielding wait only past a longer spin (GCS_SERVER_SPIN_US), 16 / 24
# unpinned threads and 8 / 16 pinned, spin baseline beside each.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06j}
mkdir -p $O
ss() { local name=$1; shift; env SS_PROF=0 SS_RINGS= "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json,sys; d=json.load(open('$O/$name.json'))
print('$name', {k: (v['us_per_call'], v['cpu_frac']) for k, v in d.items() if k.startswith('threads')})"; }
for r in 1 2; do
ss spin_$r SS_THREADS=16,24 MT_PIN=0
ss y8_$r SS_THREADS=16,24 MT_PIN=0 GCS_SERVER_WAIT=yield GCS_SERVER_SPIN_US=8
ss y12_$r SS_THREADS=16,24 MT_PIN=0 GCS_SERVER_WAIT=yield GCS_SERVER_SPIN_US=12
ss y20_$r SS_THREADS=16,24 MT_PIN=0 GCS_SERVER_WAIT=yield GCS_SERVER_SPIN_US=20
done
ss pin_spin SS_THREADS=8,16 MT_PIN=1
ss pin_y12 SS_THREADS=8,16 MT_PIN=1 GCS_SERVER_WAIT=yield GCS_SERVER_SPIN_US=12
