# Counter passes over the bench step (tools/pmc_traffic.py run) for the head-projection
# diagnosis: bash tools/pmc_hproj.sh OUTDIR
set -e
OUT=$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p1 -o run -- python tools/pmc_traffic.py run > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUSY_max TD_BUSY_avr SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d $OUT/p2 -o run -- python tools/pmc_traffic.py run > $OUT/p2.log 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/p3 -o run -- python tools/pmc_traffic.py run > $OUT/p3.log 2>&1 || true
python tools/pmc_kernels.py $OUT/p1 k_hproj > $OUT/k.txt
python tools/pmc_kernels.py $OUT/p2 k_hproj >> $OUT/k.txt || true
python tools/pmc_kernels.py $OUT/p3 k_hproj >> $OUT/k.txt || true
