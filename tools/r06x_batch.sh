set -e
OUT=gpurun_out/r06x; mkdir -p $OUT
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $PT tests/test_gpu_bf16_x.py tests/test_gpu_worklist.py -m gpu > $OUT/pytest1.log 2>&1
timeout -k 10 600 $PT tests/test_gpu_stack_parity.py -k "cfg5 or bf16" -m gpu > $OUT/pytest2.log 2>&1
HSG_AB_CONFIG=cfg5 HSG_AB_DTYPE=bf16 HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so timeout -k 10 400 python -u tools/ab.py '' 'HSG_FFN_BF16_X=0' > $OUT/ab_cfg5_bf16.txt 2>&1
for c in "cfg5 bf16" "cfg5 f32" "cfg5 bf16"; do set -- $c; timeout -k 10 240 python -u bench.py --config $1 --dtype $2 --no-cpu-baseline > $OUT/bench_$1_$2.json 2> $OUT/bench_$1_$2.err; cp $OUT/bench_$1_$2.json $OUT/bench_$1_$2_$RANDOM.json; done
echo done
