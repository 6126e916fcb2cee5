#!/bin/bash
# Round 6: the N > 1 bench flow rehearsed on one GPU (2 ranks, gloo for the
# timing collectives only; RCCL refuses two ranks on one device).
set -o pipefail
O=gpurun_out/${R06_OUT:-r06h}
mkdir -p $O
GCS_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 \
    > $O/bench_n2.json 2> $O/bench_n2.err || { tail -30 $O/bench_n2.err; exit 1; }
wc -c $O/bench_n2.json
python -c "
import json; d=json.loads(open('$O/bench_n2.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['roofline']['frac'], d['roofline']['traffic'], d['per_gpu'])"
