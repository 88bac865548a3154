# Round-4 batch for the short-row slab reduce and the paired dT pass: its GPU tests (+ the stack / model
# parity suites that now run it), an in-process A/B against the dst + src pair
# (HSG_GAT_MERGED=0), the kernel-trace profile of replayed cfg2 steps, a bench line.
# usage (repo root, via gpurun): bash tools/gpu_r04d.sh <tag> [ab variants...]
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gat.py tests/test_gpu_gemm.py tests/test_gpu_ops.py \
  tests/test_gpu_stack_parity.py tests/test_gpu_model.py -m gpu > $OUT/pytest.log 2>&1
if [ $# -gt 0 ]; then
  HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 400 python -u tools/ab.py "$@" > $OUT/ab.txt 2>&1
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/step -o step -- python tools/step_profile.py run > $OUT/step_run.log 2>&1
python tools/step_profile.py parse $(ls $OUT/step/*/step_kernel_trace.csv $OUT/step/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_kernels.txt
rm -rf $OUT/step
timeout -k 10 400 python -u bench.py --cpu-steps 1 > $OUT/bench.json 2> $OUT/bench.err
echo done
