#!/bin/bash
# Round 6: the whole GPU suite (per-test device check in conftest), smoke,
# then the default bench line and its extras file.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06a}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cp profiles/bench_extras_last.json $O/bench_extras.json
wc -c $O/bench.json
