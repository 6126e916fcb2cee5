#!/bin/bash
# Round 5: thread scaling with each worker pinned to one CPU (MT_PIN=1, as mTCP
# pins its threads) against unpinned, shipped grid, twice each.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05pin}
mkdir -p $O
for r in 1 2; do
  SS_PROF=0 SS_THREADS=1,8,12,16 SS_RINGS=4x4 MT_PIN=1 timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_pin_r$r.json 2> $O/ss_pin_r$r.err || exit 1
  SS_PROF=0 SS_THREADS=1,8,12,16 SS_RINGS=4x4 timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_nopin_r$r.json 2> $O/ss_nopin_r$r.err || exit 1
done
