# Round-4 dev A/B by kernel traces: rocprofv3 traces of replayed cfg2 steps on the dev
# library under each environment variant ("" = defaults, "VAR=v,VAR2=w"), alternated
# twice; per-kernel averages over many launches land in <tag>/step_<i>_<round>.txt.
# usage (repo root, via gpurun): [AB_CFG=cfg5 AB_DTYPE=bf16] bash tools/gpu_trace_ab.sh <tag> <variant>...
set -e
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so
for r in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    echo "$i: $v" > $OUT/variant_$i.txt
    ( for kv in ${v//,/ }; do export "$kv"; done
      HSG_PROFILE_DTYPE=${AB_DTYPE:-f32} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/s_${i}_$r -o step -- python tools/step_profile.py run ${AB_CFG:-cfg2} > $OUT/run_${i}_$r.log 2>&1 )
    python tools/step_profile.py parse $(ls $OUT/s_${i}_$r/*/step_kernel_trace.csv $OUT/s_${i}_$r/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_${i}_$r.txt
    rm -rf $OUT/s_${i}_$r
  done
done
echo done
