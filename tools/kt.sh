# Kernel-trace stats of a dev timing script: bash tools/kt.sh <tag> <script.py> [args...]
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python "$@" > $OUT/run.log 2>&1
cp $(ls $OUT/kt/*/kt_kernel_stats.csv $OUT/kt/kt_kernel_stats.csv 2>/dev/null | head -1) $OUT/kernel_stats.csv
rm -rf $OUT/kt
echo done
