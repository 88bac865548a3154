# Round-4 dev: the persistent LayerNorm forward (k_ln_fwd4p) -- bitwise test against
# k_ln_fwd4 on the dev library, then the in-step A/B of its grid by kernel traces.
set -e
mkdir -p gpurun_out/$1
HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread tests/test_gpu_ffn.py -k ln_fwd_persistent -p no:cacheprovider > gpurun_out/$1/pytest.log 2>&1
bash tools/gpu_trace_ab.sh $1 "HSG_LN_FWDP=0" "" "HSG_LN_FWDP=768" "HSG_LN_FWDP=1536"
