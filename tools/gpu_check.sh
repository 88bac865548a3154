# One GPU call: the full -m gpu suite, smoke(), and the default bench line.
# usage (repo root, via gpurun): bash tools/gpu_check.sh <tag>
set -e
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
