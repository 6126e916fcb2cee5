#!/bin/bash
# Round 5: descriptor / header prefetch A/B (kbench lro: k_gro NXP, rooms DPF).
set -o pipefail
O=gpurun_out/${R05_OUT:-r05u}
mkdir -p $O
KB_ONLY="${KB_ONLY:-k_gro|rooms|fixed stride 2048|D2D}" timeout -k 10 400 ./tools/kbench lro 1048576 ${KB_ROUNDS:-9} > $O/kbench_pf.log 2>&1 || exit 1
