set -e
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc/p1 -o run -- python tools/pmc_traffic.py run > gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/p2 -o run -- python tools/pmc_traffic.py run > gpurun_out/pmc/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_BUSY_avr --output-format csv -d gpurun_out/pmc/p3 -o run -- python tools/pmc_traffic.py run > gpurun_out/pmc/p3.log 2>&1
python tools/pmc_kernels.py gpurun_out/pmc/p1 gat hproj ln_ ffn_small > gpurun_out/pmc/k1.txt
python tools/pmc_kernels.py gpurun_out/pmc/p2 gat hproj ln_ ffn_small > gpurun_out/pmc/k2.txt
python tools/pmc_kernels.py gpurun_out/pmc/p3 gat hproj ln_ ffn_small > gpurun_out/pmc/k3.txt
