# Round-4 batch: the whole -m gpu suite against the DEV library (the variant tests that
# skip on the product library run here), then bench lines for every single-GPU
# configuration in both GEMM modes (product library).
# usage (repo root, via gpurun): bash tools/gpu_r04j.sh <tag>
set -e
OUT=gpurun_out/${1:-r04j}
mkdir -p $OUT
HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest_dev.log 2>&1
for c in "cfg2 f32" "cfg2 bf16" "cfg4 f32" "cfg4 bf16" "cfg5 f32" "cfg5 bf16"; do
  set -- $c
  timeout -k 10 240 python -u bench.py --config $1 --dtype $2 --no-cpu-baseline > $OUT/bench_$1_$2.json 2> $OUT/bench_$1_$2.err
done
echo done
