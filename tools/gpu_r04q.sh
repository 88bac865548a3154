# Round-4 batch: the narrow one-pass edge backward on a grid sized by its wave groups --
# parity (edge, stack, model tests on the product library), then trace A/B against the
# source grid (HSG_SRCG_GRID=0, dev library).
# usage (repo root, via gpurun): bash tools/gpu_r04q.sh <tag>
set -e
OUT=gpurun_out/${1:-r04q}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_elug.py \
  tests/test_gpu_gat.py tests/test_gpu_stack_parity.py tests/test_gpu_model.py -m gpu > $OUT/pytest.log 2>&1
bash tools/gpu_trace_ab.sh ${1:-r04q}/ab '' 'HSG_SRCG_GRID=0'
echo done
