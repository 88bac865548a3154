# Per-kernel step profile of one config / GEMM dtype: bash tools/prof_cfg.sh TAG CONFIG DTYPE
set -e
TAG=$1; CFG=$2; DT=$3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
HSG_PROFILE_DTYPE=$DT timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$TAG -o step -- python tools/step_profile.py run $CFG > gpurun_out/$TAG.log 2>&1
python tools/step_profile.py parse $(ls gpurun_out/$TAG/*/step_kernel_trace.csv gpurun_out/$TAG/step_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/step_$TAG.txt
rm -rf gpurun_out/$TAG
