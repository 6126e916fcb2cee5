#!/bin/bash
# Round 5: C3 stream kernel with the next generation's descriptors read ahead
# (DPF), and the shipped LRO (NXP) against round 3's k_gro.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05x}
mkdir -p $O
KB_ONLY="launch_|DPF" timeout -k 10 400 ./tools/kbench imix 4194304 ${KB_ROUNDS:-9} > $O/kbench_imix_dpf.log 2>&1 || exit 1
KB_ONLY="gro (launch|shipped r03|D2D" timeout -k 10 300 ./tools/kbench lro 1048576 ${KB_ROUNDS:-9} > $O/kbench_lro_ship.log 2>&1 || exit 1
