set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 ./tools/kbench 1500 1048576 15 > gpurun_out/kbench16_1500.log 2>&1 && \
timeout -k 10 200 ./tools/kbench 1500 4194304 7 > gpurun_out/kbench16_1500_4M.log 2>&1
echo "exit $?"
