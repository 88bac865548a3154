# One GPU call for several dev checks: selected -m gpu tests, an optional GEMM plan
# sweep (PLANS env), and an optional in-process A/B of env variants.
# usage (repo root, via gpurun): PLANS=27,43 KEXPR="a or b" bash tools/gpu_multi.sh <tag> "<test files>" [ab variants...]
set -e
TAG=$1; shift
TESTS=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $OUT/pytest.log 2>&1
fi
if [ -n "$PLANS" ]; then
  ROUNDS=${ROUNDS:-3} timeout -k 10 300 python -u tools/gemm5_sweep.py > $OUT/sweep.log 2>&1
fi
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u tools/ab.py "$@" > $OUT/ab.txt 2>&1
fi
echo done
