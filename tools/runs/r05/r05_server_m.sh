#!/bin/bash
# Round 5: where post -> done goes at many threads (wait before the GPU sees a
# request / GPU span / after), shipped grid, two rounds.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05o}
mkdir -p $O
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_$name.json 2> $O/ss_$name.err; }
C="SS_THREADS=1,4,8,12,16 SS_RINGS=4x4,4x6 SS_ITERS=400"
for rep in 1 2; do
    run counters_r$rep $C || exit 1
done
