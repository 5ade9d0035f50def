#!/bin/bash
# r03 first GPU call: stream-creation A/B and the 2-rank rehearsal of the N>1 bench path
# (gloo, both ranks on the one GPU; torchrun starts before any GPU call).  Each GPU step has its own limit.
OUT=gpurun_out/r03_probe1
mkdir -p $OUT
timeout -k 10 300 python -u tools/stream_ab.py --steps 10 > $OUT/stream_ab.log 2>&1
rc=$?; tail -12 $OUT/stream_ab.log; [ $rc -eq 0 ] || exit $rc
SMC_DIST_BACKEND=gloo SMC_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 \
    > $OUT/dist2_gloo_bench.log 2>&1
rc=$?; tail -3 $OUT/dist2_gloo_bench.log; exit $rc
