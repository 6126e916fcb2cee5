#!/bin/bash
# Round 5: the server tests under leader-only polling (A/B mode must stay exact).
set -o pipefail
O=gpurun_out/${R05_OUT:-r05c}
mkdir -p $O
GCS_SERVER_POLL=leader timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_host.py tests/test_gpu_mt.py > $O/pytest_server_leader.log 2>&1 || exit 1
