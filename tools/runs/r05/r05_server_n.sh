#!/bin/bash
# Round 5: records as one 64 B line per pass: server tests, then where
# post -> done goes (two rounds).
set -o pipefail
O=gpurun_out/${R05_OUT:-r05p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_host.py tests/test_plugin_faults.py tests/test_gpu_mt.py tests/test_plugin.py > $O/pytest_server.log 2>&1 || exit 1
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_$name.json 2> $O/ss_$name.err; }
C="SS_THREADS=1,4,8,12,16 SS_RINGS=4x4,4x6 SS_ITERS=400"
for rep in 1 2; do
    run lines_r$rep $C || exit 1
done
