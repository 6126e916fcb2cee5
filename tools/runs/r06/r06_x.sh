#!/bin/bash
# Round 6, final build: smoke, the default bench line, then the profile
# collection (profiles/collect.sh r06).  The GPU suite on this build: r06w.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06x}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cp profiles/bench_extras_last.json $O/bench_extras.json
wc -c $O/bench.json
bash profiles/collect.sh r06
