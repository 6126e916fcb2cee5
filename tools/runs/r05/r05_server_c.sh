#!/bin/bash
# Round 5: burst-server lateness per block, slow and torn polls; the shipped
# (unprofiled) grid's per-call times beside.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05c}
mkdir -p $O
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_$name.json 2> $O/ss_$name.err
}
run dev_auto SS_THREADS=1,8,12,16 SS_RINGS=4x1,4x4,4x6 || exit 1
run dev_noprof SS_PROF=0 SS_THREADS=1,8,12,16 SS_RINGS=4x1,4x4,4x6 || exit 1
run host_noprof SS_PROF=0 GCS_SERVER_MAILBOX=host SS_THREADS=1,8,12,16 SS_RINGS=4x4 || exit 1
run dev_leader GCS_SERVER_POLL=leader SS_THREADS=1,8,12,16 SS_RINGS=4x1,4x4,4x6 || exit 1
run dev_leader_noprof SS_PROF=0 GCS_SERVER_POLL=leader SS_THREADS=1,8,12,16 SS_RINGS=4x1,4x4,4x6 || exit 1
