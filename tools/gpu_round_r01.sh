set -e
mkdir -p gpurun_out/r01
timeout -k 10 700 python -m pytest tests -m gpu -q -x > gpurun_out/r01/pytest_gpu.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r01/pmc_fetch -o run -- python tools/pmc_traffic.py run > gpurun_out/r01/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r01/pmc_write -o run -- python tools/pmc_traffic.py run > gpurun_out/r01/pmc_write.log 2>&1
python tools/pmc_traffic.py parse gpurun_out/r01/pmc_fetch gpurun_out/r01/pmc_write gpurun_out/r01/r01_pmc_traffic.json
cp gpurun_out/r01/r01_pmc_traffic.json profiles/r01_pmc_traffic.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01/trace -o bench -- python bench.py > gpurun_out/r01/bench_prof.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r01/bench.json 2> gpurun_out/r01/bench.err
