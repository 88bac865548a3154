# One GPU call: parity tests, kernel trace of bench.py, PMC traffic passes, plain bench.
# usage (from the repo root, via gpurun): bash tools/gpu_round.sh <tag> [tests|bench|all]
set -e
TAG=${1:-r01}
WHAT=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python bench.py --no-cpu-baseline > $OUT/bench_prof.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python tools/pmc_traffic.py run > $OUT/pmc_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python tools/pmc_traffic.py run > $OUT/pmc_write.log 2>&1
  python tools/pmc_traffic.py parse $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json
fi
echo done
