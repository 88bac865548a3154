# Round-4 batch: rocprofv3 kernel traces of replayed cfg2 steps on the dev library with
# the S2W forward's one-level (default) and two-level (HSG_GAT_FWD_PF=2) prefetch,
# alternated twice, for per-kernel averages over many launches.
# usage (repo root, via gpurun): bash tools/gpu_r04n.sh <tag>
set -e
OUT=gpurun_out/${1:-r04n}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so
for r in 1 2; do
  for pf in 1 2; do
    HSG_GAT_FWD_PF=$pf timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/s_${pf}_$r -o step -- python tools/step_profile.py run > $OUT/run_${pf}_$r.log 2>&1
    python tools/step_profile.py parse $(ls $OUT/s_${pf}_$r/*/step_kernel_trace.csv $OUT/s_${pf}_$r/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_pf${pf}_$r.txt
    rm -rf $OUT/s_${pf}_$r
  done
done
echo done
