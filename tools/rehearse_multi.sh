#!/bin/bash
# Rehearse bench.py's N > 1 path on a 1-GPU box: N ranks share cuda:0 and
# exchange over gloo (CUDA tensors); RCCL refuses two ranks on one device.
# usage (via gpurun): bash tools/rehearse_multi.sh TAG [N] [keys_log2]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}; N=${2:-2}; KL=${3:-22}
OUT=$R/gpurun_out/multi_$TAG
mkdir -p $OUT
cd $R
for w in c2 c5; do
  SHM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) \
    bench.py --gpus $N --steps 5 --warmup 2 --keys-log2 $KL --workload $w \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -40 $OUT/bench_$w.err; exit 1; }
  cat $OUT/bench_$w.json
done
