#!/bin/bash
# Round 5: rooms walk variants (occupancy-forced, software-pipelined) against
# the shipped k_desc<32,3>, interleaved then blocked.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05p2}
mkdir -p $O
KB_ONLY="rooms verify|rooms fill" timeout -k 10 400 ./tools/kbench lro 1048576 9 > $O/kbench_rooms_i.log 2>&1 || exit 1
KB_BLOCKED=1 KB_ONLY="rooms verify|rooms fill" timeout -k 10 400 ./tools/kbench lro 1048576 9 > $O/kbench_rooms_b.log 2>&1 || exit 1
