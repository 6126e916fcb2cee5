#!/bin/bash
# Round 6: full suite + smoke + bench on the fused-step / one-launch hybrid
# build, then the C4 shard with and without the hybrid write-back.
set -o pipefail
export R06_OUT=${R06_OUT:-r06f}
bash tools/runs/r06/r06_full.sh || exit 1
O=gpurun_out/$R06_OUT
c4() { local name=$1; shift; env "$@" timeout -k 10 180 python -u -c "
import json, torch, bench
from mtcp_amd import gpucsum
ctx = gpucsum.Context(0)
torch.cuda.set_stream(torch.cuda.Stream())
r = bench.c4_shard(ctx, torch, 20, 3, 1.0)
ctx.close()
print(json.dumps(r))" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
python -c "
import json; d=json.load(open('$O/$name.json'))
print('$name', round(d['ms_per_step'],4), 'step', round(d['step_kernel_ms'],4), round(d['roofline']['frac'],4), 'fill', round(d['compute_ms'],4), round(d['compute_frac'],4), 'verify', round(d['verify_ms'],4))"; }
for r in 1 2; do
c4 c4_default_$r
c4 c4_off_$r GCS_TX_HYBRID=off
done
