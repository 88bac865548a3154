# PMC passes over one GEMM shape (dev): bash tools/pmc_gemm.sh OUTDIR M N K a_t b_t dtype [tile]
set -e
OUT=$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/p1 -o run -- python tools/gemm_one_run.py "$@" > $OUT/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv -d $OUT/p2 -o run -- python tools/gemm_one_run.py "$@" > $OUT/p2.log 2>&1
python tools/pmc_kernels.py $OUT/p1 k_gemm > $OUT/k.txt
python tools/pmc_kernels.py $OUT/p2 k_gemm >> $OUT/k.txt
