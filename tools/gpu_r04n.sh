# Round-4 batch: rocprofv3 kernel traces of replayed cfg2 steps on the dev library with
# S2W-forward prefetch variants (HSG_GAT_FWD_PF values, default "1 2": one- and
# two-level), alternated twice, for per-kernel averages over many launches.
# usage (repo root, via gpurun): bash tools/gpu_r04n.sh <tag> [pf values...]
set -e
OUT=gpurun_out/${1:-r04n}
shift || true
PFS=${*:-1 2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export HSG_LIB_PATH=$PWD/hetersumgraph_amd/libhsg_dev.so
for r in 1 2; do
  for pf in $PFS; do
    HSG_GAT_FWD_PF=$pf timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/s_${pf}_$r -o step -- python tools/step_profile.py run > $OUT/run_${pf}_$r.log 2>&1
    python tools/step_profile.py parse $(ls $OUT/s_${pf}_$r/*/step_kernel_trace.csv $OUT/s_${pf}_$r/step_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_pf${pf}_$r.txt
    rm -rf $OUT/s_${pf}_$r
  done
done
echo done
