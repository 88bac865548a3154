# Round-4 iteration: chosen -m gpu tests, an optional in-process A/B of dev switches
# on the dev library (libhsg_dev.so), the kernel-trace profile of replayed cfg2 steps
# and a default bench line (product library).
# usage (repo root, via gpurun): bash tools/gpu_r04.sh <tag> "<pytest args>" <bench 0|1> [ab variants...]
set -e
TAG=$1; TESTS=$2; BENCH=${3:-1}; shift 3 || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
fi
if [ $# -gt 0 ]; then
  HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 400 python -u tools/ab.py "$@" > $OUT/ab.txt 2>&1
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/step -o step -- python tools/step_profile.py run > $OUT/step_run.log 2>&1
python tools/step_profile.py parse $(ls $OUT/step/*/step_kernel_trace.csv $OUT/step/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_kernels.txt
rm -rf $OUT/step
if [ "$BENCH" = "1" ]; then
  timeout -k 10 400 python -u bench.py --cpu-steps 1 > $OUT/bench.json 2> $OUT/bench.err
fi
echo done
