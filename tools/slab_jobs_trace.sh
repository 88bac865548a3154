# Kernel durations of every slab-reduce job of a cfg2 backward (tools/slab_jobs.py under a
# rocprofv3 kernel trace; each launch group is 3 warm-up + 20 timed launches).
# usage (repo root, via gpurun): bash tools/slab_jobs_trace.sh <outdir>
set -e
OUT=$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o slab -- python tools/slab_jobs.py > $OUT/slab_jobs.log 2>&1
python - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
f = (glob.glob(out + "/t/*/slab_kernel_trace.csv") + glob.glob(out + "/t/slab_kernel_trace.csv"))[0]
rows = [r for r in csv.DictReader(open(f)) if "slab_reduce" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
g = [int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) for r in rows]
with open(out + "/slab_jobs_kernels.txt", "w") as fo:
    # the first launch is the step's own; then groups of 23
    fo.write(f"step launch: {d[0]:.2f} us grid {g[0]}\n")
    for i in range(1, len(d), 23):
        seg = d[i + 3:i + 23]
        if seg:
            fo.write(f"group {(i - 1) // 23:2d}: grid {g[i]:8d}  {sum(seg) / len(seg):7.2f} us\n")
PY
rm -rf $OUT/t
