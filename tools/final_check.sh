# Round-end check on the GPU box: GPU tests, smoke, bench (N=1) and the N=2
# flow rehearsed on one GPU (gloo timing collectives, GCS_BENCH_DEVICE=0).
set -e
mkdir -p gpurun_out/final
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1
timeout -k 10 240 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
GCS_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo > gpurun_out/final/bench_n2_rehearsal.json 2> gpurun_out/final/bench_n2.err
