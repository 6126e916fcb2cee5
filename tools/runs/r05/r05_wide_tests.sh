#!/bin/bash
# Round 5: the WIDE LRO path (windows > 64): LRO parity tests, 150 random
# stream/LRO cases against the oracle, the kbench A/B with output checks.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05wide}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lro.py > $O/pytest_lro.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/stress_stream.py 150 > $O/stress_150.json 2> $O/stress_150.err || exit 1
KB_ONLY="w256|shipped r03|512 threads" timeout -k 10 400 ./tools/kbench lro 1048576 9 > $O/kbench_wide_i.log 2>&1 || exit 1
KB_BLOCKED=1 KB_ONLY="w256|shipped r03|512 threads" timeout -k 10 400 ./tools/kbench lro 1048576 9 > $O/kbench_wide_b.log 2>&1 || exit 1
