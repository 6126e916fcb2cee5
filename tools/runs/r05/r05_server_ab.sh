#!/bin/bash
# Round 5: burst-server phase profile and mailbox / acquire / hot-window A/B
# (tools/server_scaling.py), after the server's GPU tests.  Output under $O.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_host.py tests/test_plugin_faults.py tests/test_gpu_mt.py > $O/pytest_server.log 2>&1 || exit 1
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_$name.json 2> $O/ss_$name.err
}
run dev_auto GCS_SERVER_MAILBOX=device || exit 1
run dev_none GCS_SERVER_MAILBOX=device GCS_SERVER_ACQUIRE=none || exit 1
run dev_auto_hot GCS_SERVER_MAILBOX=device GCS_SERVER_HOT_US=5000 GCS_SERVER_HOT_MAX_US=5000 || exit 1
run host_auto GCS_SERVER_MAILBOX=host || exit 1
