# Round-4 dev: slab reduce without the clamped duplicate row loads (HSG_SLAB_PRED=1) --
# bitwise test on the dev library, then the in-step A/B by kernel traces.
set -e
mkdir -p gpurun_out/$1
HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread tests/test_gpu_gemm.py -k "slab_reduce" -p no:cacheprovider > gpurun_out/$1/pytest.log 2>&1
bash tools/gpu_trace_ab.sh $1 "" "HSG_SLAB_PRED=1"
