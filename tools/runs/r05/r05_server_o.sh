#!/bin/bash
# Round 5: with the records as whole lines, the counting grid against the plain
# one (three rounds), then the single-thread burst probes.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05q}
mkdir -p $O
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_$name.json 2> $O/ss_$name.err; }
C="SS_THREADS=1,8,12,16 SS_RINGS=4x4,4x6 SS_ITERS=400"
for rep in 1 2 3; do
    run counters_r$rep $C || exit 1
    run plain_r$rep SS_PROF=0 $C || exit 1
done
timeout -k 10 240 python -u tools/tx_async_probe.py > $O/tx_async_probe.json 2> $O/tx_async_probe.err || exit 1
timeout -k 10 240 python -u tools/rx_async_probe.py > $O/rx_async_probe.json 2> $O/rx_async_probe.err || exit 1
