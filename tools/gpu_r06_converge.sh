#!/bin/bash
# round 6: convergence records after the stored-state aliasing (C3, C4 every shape, C5)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r06_converge_probe.jsonl
sp=""
for s in 0 1 2 3 4; do sp="$sp env=market,lanes=8192,k=8,seed=$s,eval_every=125,n_eval=100"; done
for s in 0 1 2 3 4; do sp="$sp env=market,lanes=8192,k=8,seed=$s,eval_every=125,n_eval=100,sg=1"; done
for s in 0 1 2 3 4 5 6 7; do sp="$sp env=market,lanes=1,k=1,steps=96000,seed=$s,eval_every=1000,n_eval=100"; done
for s in 0 1 2 3 4 5 6 7 8 9; do sp="$sp env=dice_sh_a,algo=TD3,loss=MSE,k=8,seed=$s"; done
for s in 0 1 2 3 4 5 6 7 8 9; do sp="$sp env=gbm,algo=TD3,loss=MSE,k=8,ms=5,seed=$s"; done
timeout -k 10 700 python -u tools/converge_batch.py $O $sp && \
timeout -k 10 400 python -u tools/probe/market_single.py gpurun_out/r06_market_single.jsonl 100000 0,1,2,3,4
