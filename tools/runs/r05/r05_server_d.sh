#!/bin/bash
# Round 5: the server with the exit command and profile sums in device memory
# (no PCIe read per poll at all): tests, then scaling, profiled and not.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_host.py tests/test_plugin_faults.py tests/test_gpu_mt.py > $O/pytest_server.log 2>&1 || exit 1
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_$name.json 2> $O/ss_$name.err
}
run dev_noprof SS_PROF=0 SS_THREADS=1,8,12,16 SS_RINGS=4x1,4x4,4x6 || exit 1
run dev_prof SS_THREADS=1,8,12,16 SS_RINGS=4x1,4x4,4x6 || exit 1
run host_noprof SS_PROF=0 GCS_SERVER_MAILBOX=host SS_THREADS=1,8,12,16 SS_RINGS=4x4,4x6 || exit 1
run dev_noprof2 SS_PROF=0 SS_THREADS=1,8,12,16 SS_RINGS=4x1,4x4,4x6 || exit 1
