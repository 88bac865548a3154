# Round-4 batch: DPP wave / group sums (hsg_wave.h) and the software-pipelined LayerNorm
# backward -- the GPU tests of every kernel they touch (edge, LayerNorm, narrow FFN,
# GEMM epilogues; the GEMM file also against the dev library, whose LayerNorm-epilogue
# test is bitwise), stack / model parity, the step profile and a bench line.
# usage (repo root, via gpurun): bash tools/gpu_r04l.sh <tag>
set -e
OUT=gpurun_out/${1:-r04l}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_ffn.py \
  tests/test_gpu_elug.py tests/test_gpu_ops.py tests/test_gpu_gat.py tests/test_gpu_gemm.py tests/test_gpu_dropout_masks.py \
  tests/test_gpu_stack_parity.py tests/test_gpu_model.py tests/test_gpu_stack.py -m gpu > $OUT/pytest.log 2>&1
HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 300 python -u -m pytest -x -q --timeout 150 \
  --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_ops.py -m gpu > $OUT/pytest_dev.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/step -o step -- python tools/step_profile.py run > $OUT/step_run.log 2>&1
python tools/step_profile.py parse $(ls $OUT/step/*/step_kernel_trace.csv $OUT/step/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_kernels.txt
rm -rf $OUT/step
timeout -k 10 400 python -u bench.py --cpu-steps 1 > $OUT/bench.json 2> $OUT/bench.err
echo done
