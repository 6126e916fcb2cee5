#!/bin/bash
# Round 5: rooms-hint parity tests and the c2_rooms bench extra alone.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -k "sparse_rooms" > $O/pytest_rooms.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
from mtcp_amd import gpucsum
ctx = gpucsum.Context(0)
s = torch.cuda.Stream(); torch.cuda.set_stream(s)
print(json.dumps(bench.c2_rooms(ctx, torch)))
" > $O/c2_rooms.json 2> $O/c2_rooms.err || exit 1
