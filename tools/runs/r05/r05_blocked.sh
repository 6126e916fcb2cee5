#!/bin/bash
# Round 5: blocked A/B (each variant's rounds back to back, KB_BLOCKED=1), so
# that no variant runs behind another's write-back: LRO read-ahead and rooms.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05y}
mkdir -p $O
KB_BLOCKED=1 KB_ONLY="gro (launch|shipped r03|DIAG|NXP 1024 PF 16|rooms|fixed stride 2048" timeout -k 10 400 ./tools/kbench lro 1048576 ${KB_ROUNDS:-9} > $O/kbench_blocked.log 2>&1 || exit 1
KB_BLOCKED=1 KB_ONLY="launch_|DPF" timeout -k 10 400 ./tools/kbench imix 4194304 ${KB_ROUNDS:-9} > $O/kbench_imix_blocked.log 2>&1 || exit 1
