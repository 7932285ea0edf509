set -o pipefail
cd "$GRAFT_REPO_ROOT"
P=tools/probe/market_sweep.py
O=gpurun_out/r05_market_sweepB.jsonl
timeout -k 10 300 python -u $P $O "1:1" 3,4,5,6,7,8,9,10,11,12 > gpurun_out/r05_sweepB1.log 2>&1 &&
timeout -k 10 200 python -u $P $O "1:1:0:0:1" 0,1,2,3,4,5 > gpurun_out/r05_sweepB2.log 2>&1 &&
timeout -k 10 300 python -u $P $O "8192:8:67108864,512:1:67108864" 0,1,2 > gpurun_out/r05_sweepB3.log 2>&1 &&
timeout -k 10 200 python -u $P $O "8192:8,8192:8:0:0:1" 3,4,5,6,7 > gpurun_out/r05_sweepB4.log 2>&1
echo rc=$?
