set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu8.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu8.log
grep -q "rc=0" gpurun_out/pytest_gpu8.log && \
timeout -k 10 200 ./tools/kbench 1500 1048576 15 > gpurun_out/kbench8_1500.log 2>&1 && \
timeout -k 10 200 ./tools/kbench 64 1048576 15 > gpurun_out/kbench8_64.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 1 > gpurun_out/bench8.json 2> gpurun_out/bench8.err
echo "exit $?"
