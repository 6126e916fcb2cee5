#!/bin/bash
# Round 5: the C3 fill's write set three ways -- 64 B sectors
# at the IMIX offsets, their whole 128 B lines, the same bytes contiguous --
# beside the shipped fill, blocked and interleaved.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05c}
mkdir -p $O
KB_ONLY="write|compute stream 7 waves|verify  stream U8 R8K occ7" timeout -k 10 300 tools/kbench imix > $O/kbench_imix_writes.log 2>&1 || exit 1
KB_BLOCKED=1 KB_ONLY="write|compute stream 7 waves" timeout -k 10 300 tools/kbench imix > $O/kbench_imix_writes_blocked.log 2>&1 || exit 1
