#!/bin/bash
# Round 5: LRO windows of 256 in the FLAT form (WIDE) against the run-per-wave
# kernel, blocked and interleaved, outputs compared.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05w256}
mkdir -p $O
KB_BLOCKED=1 KB_ONLY="w256|shipped r03" timeout -k 10 400 ./tools/kbench lro 1048576 9 > $O/kbench_w256_b.log 2>&1 || exit 1
KB_ONLY="w256|shipped r03" timeout -k 10 400 ./tools/kbench lro 1048576 9 > $O/kbench_w256_i.log 2>&1 || exit 1
