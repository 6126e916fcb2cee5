#!/bin/bash
# Round 6: the final build's GPU suite again on another box (stability), then
# the N = 2 torchrun flow rehearsed on the one GPU (gloo for the timing
# collectives), as the driver's scaling run starts it.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06v}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
GCS_BENCH_DEVICE=0 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 \
    --dist-backend gloo > $O/bench_n2.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_n2.json').read().strip().splitlines()[-1]); print('n2 rehearsal', d['value'], d['n_gpus'], d['ms_per_step'], [p['gpkt_per_s'] for p in d['per_gpu']])"
