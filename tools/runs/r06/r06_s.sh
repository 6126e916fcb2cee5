#!/bin/bash
# Round 6: the bench's C4 side line (2.02-2.03 ms per step) against the same
# step alone (1.94-1.95 ms, r06r): the full bench with and without the CPU
# baseline that runs just before it.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06s}
mkdir -p $O
for c in 0 8; do
timeout -k 10 420 python -u bench.py --cpu-seconds $c > $O/bench_cpu$c.json 2> $O/bench_cpu$c.err || { tail -5 $O/bench_cpu$c.err; exit 1; }
cp profiles/bench_extras_last.json $O/bench_extras_cpu$c.json
python -c "
import json; d=json.load(open('$O/bench_cpu$c.json')); s=d['side']; print('cpu=$c', d['value'], {k: s[k] for k in s if k.startswith('c4') or k.startswith('c2')})"
done
