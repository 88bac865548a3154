# One GPU iteration: selected -m gpu tests, an in-process A/B of env variants, and a
# kernel-trace profile of replayed cfg2 steps.
# usage (repo root, via gpurun): bash tools/gpu_iter.sh <tag> "<pytest -k expr or files>" [ab variants...]
set -e
TAG=$1; shift
TESTS=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
fi
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u tools/ab.py "$@" > $OUT/ab.txt 2>&1
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/step -o step -- python tools/step_profile.py run > $OUT/step_run.log 2>&1
python tools/step_profile.py parse $(ls $OUT/step/*/step_kernel_trace.csv $OUT/step/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_kernels.txt
rm -rf $OUT/step
echo done
