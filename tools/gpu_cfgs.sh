# One GPU call: GEMM/model parity (incl. the bf16 mode) and bench lines for every
# single-GPU configuration.  usage (repo root, via gpurun): bash tools/gpu_cfgs.sh <tag>
set -e
TAG=${1:-cfgs}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_model.py -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
for c in "cfg2 f32" "cfg2 bf16" "cfg4 f32" "cfg4 bf16" "cfg5 f32" "cfg5 bf16"; do
  set -- $c
  timeout -k 10 240 python -u bench.py --config $1 --dtype $2 --no-cpu-baseline > $OUT/bench_$1_$2.json 2> $OUT/bench_$1_$2.err
done
echo done
