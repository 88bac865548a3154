# PMC passes over one GEMM shape (x W1^T of the S2W FFN): MFMA busy, waits, LDS conflicts.
set -e
OUT=gpurun_out/gpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python tools/gemm_one.py 19200 512 300 0 1 20 > $OUT/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAIT_INST_LDS --output-format csv -d $OUT/p2 -o run -- python tools/gemm_one.py 19200 512 300 0 1 20 > $OUT/p2.log 2>&1
echo done
