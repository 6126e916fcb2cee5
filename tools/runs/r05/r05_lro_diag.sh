#!/bin/bash
# Round 5: LRO diagnostics in kbench (shipped k_gro FLAT vs variants), then the
# c2_rooms bench extra (rooms hint vs the fixed-stride kernels on the same rooms).
set -o pipefail
O=gpurun_out/${R05_OUT:-r05t}
mkdir -p $O
KB_ONLY="${KB_ONLY:-k_gro|D2D}" timeout -k 10 300 ./tools/kbench lro 1048576 ${KB_ROUNDS:-9} > $O/kbench_lro.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
from mtcp_amd import gpucsum
ctx = gpucsum.Context(0)
s = torch.cuda.Stream(); torch.cuda.set_stream(s)
print(json.dumps(bench.c2_rooms(ctx, torch)))
" > $O/c2_rooms.json 2> $O/c2_rooms.err || exit 1
