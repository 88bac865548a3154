# Kernel-trace timing of the W2S head-projection forward per variant of one env var.
# usage: bash tools/hproj_trace.sh VAR v1 v2 ...
set -e
OUT=gpurun_out/hptr
mkdir -p $OUT
VAR=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  export $VAR=$v
  timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$VAR$v -o run -- python tools/hproj_one.py > $OUT/$VAR$v.log 2>&1
done
echo done
