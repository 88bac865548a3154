# Round evidence in one GPU call (tools/gpu_batch.sh steps): the full -m gpu suite,
# smoke(), the in-step PMC traffic and SQ counter passes, the kernel-trace profile of
# replayed steps, the per-shape FFN GEMM table, the head-projection counters, the
# rocprofv3 --stats trace of bench.py and the default bench line.
# usage (repo root, via gpurun): bash tools/gpu_final.sh <tag>;  results in gpurun_out/<tag>/
set -e
bash tools/gpu_batch.sh ${1:-final} tests smoke traffic sq trace shapes hproj benchprof bench
