#!/bin/bash
# Round 5: rooms kernel without load guards / batch loop (upper bounds), blocked
# and interleaved, the shipped kernel at both ends.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05rs}
mkdir -p $O
KB_BLOCKED=1 KB_ONLY="rooms verify k_desc|rooms fill k_desc|fixed stride 2048" timeout -k 10 300 ./tools/kbench lro 1048576 9 > $O/kbench_rooms_safe_b.log 2>&1 || exit 1
KB_ONLY="rooms verify k_desc|rooms fill k_desc|fixed stride 2048" timeout -k 10 300 ./tools/kbench lro 1048576 9 > $O/kbench_rooms_safe_i.log 2>&1 || exit 1
