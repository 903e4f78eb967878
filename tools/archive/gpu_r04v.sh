# Round 4, GPU call V: the multi-rank bench path rehearsed on one GPU (every
# rank on cuda:0, RCCL over sockets: GSMPM_SHARE_GPU=1) with the round's
# defaults (render worker thread on rank 0, slab re-cutting), 2 and 4 ranks.
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
for n in 2 4; do
  GSMPM_SHARE_GPU=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29590 + n)) bench.py --gpus $n --steps 5 --warmup 2 > $O/slab_$n.json 2> $O/slab_$n.err || { tail -20 $O/slab_$n.err; exit 1; }
  tail -c 700 $O/slab_$n.json; echo
done
