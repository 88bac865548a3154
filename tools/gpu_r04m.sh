# Round-4 batch: the S2W forward's two-level prefetch (HSG_GAT_FWD_PF=2, dev library):
# edge / stack parity with it switched on, then an in-process A/B of the step.
# usage (repo root, via gpurun): bash tools/gpu_r04m.sh <tag>
set -e
OUT=gpurun_out/${1:-r04m}
mkdir -p $OUT
HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so HSG_GAT_FWD_PF=2 timeout -k 10 500 python -u -m pytest -x -q \
  --timeout 150 --timeout-method thread tests/test_gpu_gat.py tests/test_gpu_ops.py tests/test_gpu_stack_parity.py \
  tests/test_gpu_model.py -m gpu > $OUT/pytest_pf2.log 2>&1
HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 400 python -u tools/ab.py '' 'HSG_GAT_FWD_PF=2' \
  'HSG_GAT_FWD_PF=0' > $OUT/ab.txt 2>&1
echo done
