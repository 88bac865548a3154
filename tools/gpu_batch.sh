# One parametrised GPU batch (replaces the per-round one-off scripts).
# usage (repo root, via gpurun): bash tools/gpu_batch.sh <tag> <step>...
# results in gpurun_out/<tag>/.  Steps run in the order given; the first that fails
# ends the batch (set -e), and every GPU step has its own time limit.
#   tests                   the whole -m gpu suite (pytest_gpu.log)
#   tests=<file>[+<file>]   those test files only, -m gpu (pytest.log)
#   devtests=<file>[+...]   the same against the dev library (pytest_dev.log)
#   smoke                   __graft_entry__.smoke() (smoke.log)
#   trace                   rocprofv3 kernel trace of 100 replayed cfg2 steps (step_kernels.txt)
#   trace=<cfg>[:<dtype>]   the same on another config / GEMM dtype (step_kernels_<cfg>_<dtype>.txt)
#   ab=<v1>;<v2>;...        dev-library trace A/B of env variants ('' = defaults), alternated twice
#   abstep=<v1>;<v2>;...    dev-library in-process step-time A/B (tools/ab.py)
#   sq                      two SQ counter passes over in-step launches, incl. SQ_LDS_BANK_CONFLICT (pmc_kernels.txt)
#   traffic                 FETCH_SIZE / WRITE_SIZE passes of the roofline kernel (pmc_traffic.json)
#   shapes                  per-shape FFN GEMM table (gemm_shapes.md)
#   hproj                   head-projection counter passes (hproj/)
#   benchprof               rocprofv3 --kernel-trace --stats over bench.py (trace/, bench_prof.json)
#   bench                   the default bench line (bench.json)
#   bench=<args>            bench.py with extra arguments, '+' for spaces (bench_<n>.json)
#   cfgs                    bench lines of every single-GPU configuration, f32 and bf16 (cfgs/)
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
ROOT=$PWD
DEV=$ROOT/hetersumgraph_amd/libhsg_dev.so
PT="python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider"
first() { ls "$@" 2>/dev/null | head -1; }
nb=0
for step in "$@"; do
  echo "[$(date +%T)] $step" >> $OUT/steps.log
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 ;;
    tests=*)
      timeout -k 10 600 $PT $(echo ${step#tests=} | tr '+' ' ') -m gpu > $OUT/pytest.log 2>&1 ;;
    devtests=*)
      HSG_LIB_PATH=$DEV timeout -k 10 600 $PT $(echo ${step#devtests=} | tr '+' ' ') -m gpu > $OUT/pytest_dev.log 2>&1 ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    trace|trace=*)
      spec=${step#trace}; spec=${spec#=}; spec=${spec:-cfg2}
      cfg=${spec%%:*}; dt=f32; [ "$spec" != "$cfg" ] && dt=${spec#*:}
      tg=${cfg}_$dt
      (cd /tmp && export TMPDIR=/tmp && cd $ROOT &&
       HSG_PROFILE_DTYPE=$dt timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/step_$tg -o step -- python tools/step_profile.py run $cfg > $OUT/step_run_$tg.log 2>&1)
      python tools/step_profile.py parse $(first $OUT/step_$tg/*/step_kernel_trace.csv $OUT/step_$tg/step_kernel_trace.csv) > $OUT/step_kernels_$tg.txt
      rm -rf $OUT/step_$tg ;;
    ab=*)
      IFS=';' read -ra VS <<< "${step#ab=}"
      bash tools/gpu_trace_ab.sh $TAG/ab "${VS[@]}" ;;
    abstep=*)
      IFS=';' read -ra VS <<< "${step#abstep=}"
      HSG_LIB_PATH=$DEV timeout -k 10 500 python -u tools/ab.py "${VS[@]}" > $OUT/ab_step.txt 2>&1 ;;
    sq)
      (cd /tmp && export TMPDIR=/tmp && cd $ROOT &&
       timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT/pmc_sq1 -o run -- python tools/pmc_traffic.py run > $OUT/pmc_sq1.log 2>&1 &&
       timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc_sq2 -o run -- python tools/pmc_traffic.py run > $OUT/pmc_sq2.log 2>&1)
      python tools/pmc_kernels.py $OUT/pmc_sq1 > $OUT/pmc_kernels.txt
      python tools/pmc_kernels.py $OUT/pmc_sq2 >> $OUT/pmc_kernels.txt
      rm -rf $OUT/pmc_sq1 $OUT/pmc_sq2 ;;
    traffic)
      (cd /tmp && export TMPDIR=/tmp && cd $ROOT &&
       timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python tools/pmc_traffic.py run > $OUT/pmc_fetch.log 2>&1 &&
       timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python tools/pmc_traffic.py run > $OUT/pmc_write.log 2>&1)
      python tools/pmc_traffic.py parse $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json
      rm -rf $OUT/pmc_fetch $OUT/pmc_write ;;
    shapes)
      (cd /tmp && export TMPDIR=/tmp && cd $ROOT &&
       timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shapes -o shapes -- python tools/gemm_shapes.py run > $OUT/shapes_run.log 2>&1)
      python tools/gemm_shapes.py parse $(first $OUT/shapes/*/shapes_kernel_trace.csv $OUT/shapes/shapes_kernel_trace.csv) > $OUT/gemm_shapes.md
      rm -rf $OUT/shapes ;;
    hproj)
      bash tools/pmc_hproj.sh $OUT/hproj ;;
    benchprof)
      (cd /tmp && export TMPDIR=/tmp && cd $ROOT &&
       timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python bench.py --no-cpu-baseline --no-e2e > $OUT/bench_prof.json 2> $OUT/bench_prof.err)
      rm -f $OUT/trace/*/bench_kernel_trace.csv $OUT/trace/bench_kernel_trace.csv ;;
    bench)
      timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err ;;
    bench=*)
      nb=$((nb + 1))
      timeout -k 10 400 python -u bench.py $(echo ${step#bench=} | tr '+' ' ') > $OUT/bench_$nb.json 2> $OUT/bench_$nb.err ;;
    cfgs)
      mkdir -p $OUT/cfgs
      for c in "cfg2 f32" "cfg2 bf16" "cfg4 f32" "cfg4 bf16" "cfg5 f32" "cfg5 bf16"; do
        set -- $c
        timeout -k 10 240 python -u bench.py --config $1 --dtype $2 --no-cpu-baseline > $OUT/cfgs/bench_$1_$2.json 2> $OUT/cfgs/bench_$1_$2.err
      done ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo done
