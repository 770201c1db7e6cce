#!/bin/bash
# the bench's N > 1 path (torchrun, weak + strong scaling, training all-reduce) rehearsed on a one-GPU box:
# N ranks share cuda:0 over gloo (timings meaningless; the driver's N-GPU runs use RCCL).  The
# sharded resident dopri5 is off: N ranks' resident grids would not fit one GPU together
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
for n in ${NS:-2 4}; do
  FETODE_RESIDENT_SHARDED=0 FETODE_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 2 --train-iters 3 --no-dopri5 \
    > $O/rehearse_$n.log 2>&1
  rc=$?; echo "== N=$n rc=$rc"; tail -c 700 $O/rehearse_$n.log; echo; [ $rc -eq 0 ] || exit $rc
done
