# Round-4 dev: the vector LayerNorm backward (k_ln_bwd4p) -- tests against k_ln_bwd on
# the dev library, then the in-step A/B (kernel variant x grid cap) by kernel traces.
set -e
mkdir -p gpurun_out/$1
HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread tests/test_gpu_ffn.py -k "ln_bwd_vector or ln_fwd_persistent" -p no:cacheprovider > gpurun_out/$1/pytest.log 2>&1
bash tools/gpu_trace_ab.sh $1 "" "HSG_LN_BWDP=1" "HSG_LN_BWDP=1,HSG_LN_BWD_CAP=1024" "HSG_LN_BWDP=1,HSG_LN_BWD_CAP=1536"
