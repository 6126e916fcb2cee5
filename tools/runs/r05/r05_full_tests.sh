#!/bin/bash
# Round 5: the whole GPU suite on the current build, then smoke.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05i}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
