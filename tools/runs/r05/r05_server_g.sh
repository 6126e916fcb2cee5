#!/bin/bash
# Round 5: server blocks per CU (dynamic LDS per block: 0 = up to 4 per CU by
# VGPRs, 60 KiB = 2, 96 KiB = 1), plain and profiled, two rounds.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05g}
mkdir -p $O
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_$name.json 2> $O/ss_$name.err
}
C="SS_THREADS=1,8,16 SS_RINGS=4x4,4x6 SS_ITERS=400"
for rep in 1 2; do
    for kb in 0 60 96; do
        run plain_lds${kb}_r$rep SS_PROF=0 GCS_SERVER_LDS_KB=$kb $C || exit 1
    done
    run prof_lds96_r$rep GCS_SERVER_LDS_KB=96 $C || exit 1
done
GCS_SERVER_LDS_KB=96 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_host.py tests/test_gpu_mt.py > $O/pytest_lds96.log 2>&1 || exit 1
