#!/bin/bash
# Round 6: regions registered uncached (the grid skips the L2 invalidate for
# their frames) -- host/plugin tests, the RX split both ways, the plugin's RX
# and TX probes, the direct bursts.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_plugin.py tests/test_plugin_faults.py tests/test_plugin_shapes.py tests/test_gpu_mt.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_host.log 2>&1 || { tail -40 $O/pytest_host.log; exit 1; }
tail -2 $O/pytest_host.log
run() { local name=$1; shift; env "$@" timeout -k 10 240 python -u tools/rx_split.py > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; cat $O/$name.json; }
run rxs_reg_uc
run rxs_reg_cached GCS_REGISTER_UNCACHED=0
run rxs_reg_uc_plain GCS_SERVER_COUNTERS=0
run rxs_reg_cached_plain GCS_SERVER_COUNTERS=0 GCS_REGISTER_UNCACHED=0
timeout -k 10 300 python -u tools/rx_async_probe.py > $O/rx_async.json 2> $O/rx_async.err || { tail -5 $O/rx_async.err; exit 1; }
python -c "
import json; d=json.load(open('$O/rx_async.json'))
print({k: round(v['blocked_us_median'],2) for k,v in d.items() if isinstance(v,dict) and 'blocked_us_median' in v})"
GCS_REGISTER_UNCACHED=0 timeout -k 10 300 python -u tools/rx_async_probe.py > $O/rx_async_cached.json 2> $O/rx_async_cached.err || { tail -5 $O/rx_async_cached.err; exit 1; }
python -c "
import json; d=json.load(open('$O/rx_async_cached.json'))
print('cached', {k: round(v['blocked_us_median'],2) for k,v in d.items() if isinstance(v,dict) and 'blocked_us_median' in v})"
timeout -k 10 300 python -u tools/tx_async_probe.py > $O/tx_async.json 2> $O/tx_async.err || { tail -5 $O/tx_async.err; exit 1; }
python -c "
import json; d=json.load(open('$O/tx_async.json'))
print({k: (round(v['send_pkts_us_median'],2), round(v['burst_us_median'],2)) for k,v in d.items() if isinstance(v,dict) and 'send_pkts_us_median' in v})"
