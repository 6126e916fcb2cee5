#!/bin/bash
# Round 6: where the RX burst's blocked time goes (tools/rx_split.py, counting
# grid), acquire scope A/B; host wait policies at 8 / 16 / 24 threads.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_plugin.py tests/test_plugin_faults.py tests/test_plugin_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_host.log 2>&1 || { tail -40 $O/pytest_host.log; exit 1; }
tail -2 $O/pytest_host.log
timeout -k 10 300 python -u -c "
import json, bench
from mtcp_amd import gpucsum
print(json.dumps(bench.plugin_bursts(gpucsum)))" > $O/plugin_bursts.json 2> $O/plugin_bursts.err || { tail -5 $O/plugin_bursts.err; exit 1; }
cat $O/plugin_bursts.json
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/rx_split.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; cat $O/$name.json; }
run rxs_reg_default
run rxs_reg_agent GCS_SERVER_ACQUIRE=agent
run rxs_reg_plain GCS_SERVER_COUNTERS=0
run rxs_reg_plain_agent GCS_SERVER_COUNTERS=0 GCS_SERVER_ACQUIRE=agent
run rxs_pageable RXS_ROOMS=pageable
ss() { local name=$1; shift; env SS_PROF=0 SS_RINGS= "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json,sys; d=json.load(open('$O/$name.json'))
print('$name', {k: (v['us_per_call'], v['cpu_frac']) for k, v in d.items() if k.startswith('threads')})"; }
ss ss_spin SS_THREADS=8,16,24 MT_PIN=0
ss ss_yield SS_THREADS=8,16,24 MT_PIN=0 GCS_SERVER_WAIT=yield
ss ss_sleep SS_THREADS=8,16,24 MT_PIN=0 GCS_SERVER_WAIT=sleep
ss ss_sleep8 SS_THREADS=8,16,24 MT_PIN=0 GCS_SERVER_WAIT=sleep GCS_SERVER_SPIN_US=8
ss ss_pin_spin SS_THREADS=8,16 MT_PIN=1
ss ss_pin_yield SS_THREADS=8,16 MT_PIN=1 GCS_SERVER_WAIT=yield
ss ss_pin_sleep SS_THREADS=8,16 MT_PIN=1 GCS_SERVER_WAIT=sleep
