# Round-4 batch: rehearsal of the multi-rank bench path on the box's one GPU -- two
# ranks under torch.distributed.run with gloo (HSG_DIST_BACKEND=gloo; the JSON contract,
# doc-weighted flat exchange and max-over-ranks timing), and the world-size-1 RCCL run
# with the exchange captured in the step graph (HSG_DP_REHEARSAL=1).
# usage (repo root, via gpurun): bash tools/gpu_r04v.sh <tag>
set -e
OUT=gpurun_out/${1:-r04v}
mkdir -p $OUT
HSG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e \
  > $OUT/dist2_gloo.json 2> $OUT/dist2_gloo.err
HSG_DP_REHEARSAL=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > $OUT/dp1_rccl.json 2> $OUT/dp1_rccl.err
echo done
