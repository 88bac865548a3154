# Final-tree check in one GPU call: the full -m gpu suite, smoke(), the per-step kernel
# profile, the rocprofv3 stats of bench.py and the default bench line.
# usage (repo root, via gpurun): bash tools/gpu_quick_final.sh <tag>;  results in gpurun_out/<tag>/
set -e
OUT=gpurun_out/${1:-qfinal}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/step -o step -- python tools/step_profile.py run > $OUT/step_run.log 2>&1
python tools/step_profile.py parse $(ls $OUT/step/*/step_kernel_trace.csv $OUT/step/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_kernels.txt
rm -rf $OUT/step
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_prof.json 2> $OUT/bench_prof.err
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
