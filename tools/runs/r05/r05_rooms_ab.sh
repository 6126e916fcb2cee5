#!/bin/bash
# Round 5: k_rooms shapes (GCS_ROOMS_K) on 1M x 1500 B in 2 KiB rooms, parity first.
set -o pipefail
O=gpurun_out/${R05_OUT:-r05c}
mkdir -p $O
for k in 2 12 34; do
    GCS_ROOMS_K=$k timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
        tests/test_gpu_parity.py -k "sparse_rooms" > $O/pytest_rooms_k$k.log 2>&1 || exit 1
done
for k in 1 2 4 12 14 34 316 1; do
    GCS_ROOMS_K=$k timeout -k 10 300 python -u -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
from mtcp_amd import gpucsum
ctx = gpucsum.Context(0)
s = torch.cuda.Stream(); torch.cuda.set_stream(s)
print(json.dumps(bench.c2_rooms(ctx, torch)))
" >> $O/c2_rooms_k.jsonl 2> $O/c2_rooms_k$k.err || exit 1
done
