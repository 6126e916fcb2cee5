#!/bin/bash
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_$name.json 2> $O/ss_$name.err; }
C="SS_THREADS=1,8,16 SS_RINGS=4x4,4x6 SS_ITERS=400"
for rep in 1 2 3; do
    run plain_r$rep SS_PROF=0 $C || exit 1
    run stores_r$rep SS_PROF=0 GCS_SERVER_AB=0x1000 $C || exit 1
    run pollwait_r$rep SS_PROF=0 GCS_SERVER_AB=0x2000 $C || exit 1
    run prof_r$rep $C || exit 1
done
