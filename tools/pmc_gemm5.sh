# PMC passes over the pre-split-weight GEMM (dev): bash tools/pmc_gemm5.sh OUTDIR [KERNEL]  (plan from HSG_GEMM5)
set -e
OUT=$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/p1 -o run -- python tools/gemm5_one.py > $OUT/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/p2 -o run -- python tools/gemm5_one.py > $OUT/p2.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES --output-format csv -d $OUT/p3 -o run -- python tools/gemm5_one.py > $OUT/p3.log 2>&1 || true
python tools/pmc_kernels.py $OUT/p1 ${2:-k_gemm5} > $OUT/k.txt
python tools/pmc_kernels.py $OUT/p2 ${2:-k_gemm5} >> $OUT/k.txt
python tools/pmc_kernels.py $OUT/p3 ${2:-k_gemm5} >> $OUT/k.txt || true
