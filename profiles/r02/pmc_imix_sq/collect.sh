set -e
mkdir -p gpurun_out/pmc_imix
export KB_ONLY="desc (launch"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_imix/p1 -o p1 --output-format csv -- tools/kbench imix 4194304 3 > gpurun_out/pmc_imix/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_imix/kt -o kt --output-format csv -- tools/kbench imix 4194304 3 > gpurun_out/pmc_imix/kt.log 2>&1
