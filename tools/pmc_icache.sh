# instruction-fetch stall counters over a short C2 bench (per kernel): does the
# learn path wait on instruction fetch?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_icache
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES -d $OUT/p1 -o p1 -f csv -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 6 --warmup 2 > $OUT/p1.log 2>&1
echo P1=$?
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ -d $OUT/p2 -o p2 -f csv -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 6 --warmup 2 > $OUT/p2.log 2>&1
echo P2=$?
