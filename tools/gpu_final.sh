# Round evidence in one GPU call: the full -m gpu suite, smoke(), the in-step PMC
# traffic passes of the roofline kernel, per-kernel counters of the edge / head
# projection / FFN kernels, the kernel-trace profile of bench.py and of replayed
# steps, the per-shape FFN GEMM table, the head-projection counter passes, and the
# default bench line.
# usage (repo root, via gpurun): bash tools/gpu_final.sh <tag>;  results in gpurun_out/<tag>/
set -e
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python tools/pmc_traffic.py run > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python tools/pmc_traffic.py run > $OUT/pmc_write.log 2>&1
python tools/pmc_traffic.py parse $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json
cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT/pmc_sq1 -o run -- python tools/pmc_traffic.py run > $OUT/pmc_sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_sq2 -o run -- python tools/pmc_traffic.py run > $OUT/pmc_sq2.log 2>&1
python tools/pmc_kernels.py $OUT/pmc_sq1 > $OUT/pmc_kernels.txt
python tools/pmc_kernels.py $OUT/pmc_sq2 >> $OUT/pmc_kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/step -o step -- python tools/step_profile.py run > $OUT/step_run.log 2>&1
python tools/step_profile.py parse $(ls $OUT/step/*/step_kernel_trace.csv $OUT/step/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_kernels.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shapes -o shapes -- python tools/gemm_shapes.py run > $OUT/shapes_run.log 2>&1
python tools/gemm_shapes.py parse $(ls $OUT/shapes/*/shapes_kernel_trace.csv $OUT/shapes/shapes_kernel_trace.csv 2>/dev/null | head -1) > $OUT/gemm_shapes.md
bash tools/pmc_hproj.sh $OUT/hproj
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_prof.json 2> $OUT/bench_prof.err
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
