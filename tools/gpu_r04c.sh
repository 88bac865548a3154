# Round-4 measurement batch: in-process A/B of dev switches (libhsg_dev.so), the
# S2W-forward PMC traffic passes, the e2e train-step attribution, the kernel-trace
# profile of replayed cfg2 steps and a default bench line (product libhsg.so).
# usage (repo root, via gpurun): bash tools/gpu_r04c.sh <tag> [ab variants...]
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ $# -gt 0 ]; then
  HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 500 python -u tools/ab.py "$@" > $OUT/ab.txt 2>&1
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python tools/pmc_traffic.py run > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python tools/pmc_traffic.py run > $OUT/pmc_write.log 2>&1
python tools/pmc_traffic.py parse $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json > $OUT/pmc_parse.log 2>&1
rm -rf $OUT/pmc_fetch $OUT/pmc_write
timeout -k 10 300 python -u tools/e2e_profile.py > $OUT/e2e_profile.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/step -o step -- python tools/step_profile.py run > $OUT/step_run.log 2>&1
python tools/step_profile.py parse $(ls $OUT/step/*/step_kernel_trace.csv $OUT/step/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_kernels.txt
rm -rf $OUT/step
timeout -k 10 400 python -u bench.py --cpu-steps 1 > $OUT/bench.json 2> $OUT/bench.err
echo done
