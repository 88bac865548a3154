set -e
mkdir -p gpurun_out/g2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g2/ops.log 2>&1
timeout -k 10 120 python -u tools/gat_fwd_lpn.py > gpurun_out/g2/lpn.txt 2>&1
timeout -s KILL 60 rocprofv3 -L > gpurun_out/g2/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/g2/pmc1 -o run -- python tools/gemm_one.py 19200 512 300 0 1 20 > gpurun_out/g2/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/g2/pmc2 -o run -- python tools/gemm_one.py 19200 512 300 0 1 20 > gpurun_out/g2/pmc2.log 2>&1
echo ok
