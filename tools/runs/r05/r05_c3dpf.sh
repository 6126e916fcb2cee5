#!/bin/bash
# Round 5: C3 stream kernel, descriptors of the next generation read ahead
# (DPF), blocked A/B twice with the order reversed.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05z2}
mkdir -p $O
KB_BLOCKED=1 KB_ONLY="verify  desc|verify  stream shipped DPF" timeout -k 10 300 ./tools/kbench imix 4194304 15 > $O/kbench_c3dpf_a.log 2>&1 || exit 1
KB_ONLY="verify  desc|verify  stream shipped DPF" timeout -k 10 300 ./tools/kbench imix 4194304 15 > $O/kbench_c3dpf_i.log 2>&1 || exit 1
KB_BLOCKED=1 KB_ONLY="compute desc (launch_compute_desc, shipped) FRESH|compute stream shipped DPF" timeout -k 10 300 ./tools/kbench imix 4194304 15 > $O/kbench_c3dpf_c.log 2>&1 || exit 1
