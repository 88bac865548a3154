# Two SQ counter passes over a dev timing script: bash tools/pmc_kt.sh <tag> <filter> <script.py> [args...]
set -e
TAG=$1; shift
FILT=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p1 -o run -- python "$@" > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/p2 -o run -- python "$@" > $OUT/p2.log 2>&1
python tools/pmc_kernels.py $OUT/p1 $FILT > $OUT/k.txt
python tools/pmc_kernels.py $OUT/p2 $FILT >> $OUT/k.txt
rm -rf $OUT/p1 $OUT/p2
echo done
