# Round-end evidence in one GPU call: the full -m gpu suite, the PMC traffic passes of
# the roofline kernel, the kernel-trace profile of bench.py and the default bench line.
# usage (repo root, via gpurun): bash tools/gpu_final.sh <tag>;  results in gpurun_out/<tag>/
set -e
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python tools/pmc_traffic.py run > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python tools/pmc_traffic.py run > $OUT/pmc_write.log 2>&1
python tools/pmc_traffic.py parse $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json
cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_prof.json 2> $OUT/bench_prof.err
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
