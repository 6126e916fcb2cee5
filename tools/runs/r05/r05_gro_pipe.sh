#!/bin/bash
# Round 5: LRO phase D2 software-pipelined vs shipped, blocked and interleaved,
# the shipped kernel at both ends of the list; then the LRO parity tests.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05g2}
mkdir -p $O
KB_BLOCKED=1 KB_ONLY="shipped r03|PIPE|D2D" timeout -k 10 400 ./tools/kbench lro 1048576 9 > $O/kbench_gro_pipe_b.log 2>&1 || exit 1
KB_ONLY="shipped r03|PIPE|D2D" timeout -k 10 400 ./tools/kbench lro 1048576 9 > $O/kbench_gro_pipe_i.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lro.py > $O/pytest_lro.log 2>&1 || exit 1
