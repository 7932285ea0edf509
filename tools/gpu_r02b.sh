# Round 2: convergence sweep on Dice_SH_INSURED / coin / dice (K, replay size, precision).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/converge_k.jsonl
rm -f $OUT
for cfg in ${CFGS:-"dice_sh 8 bf16 1048576" "dice_sh 8 fp32 1048576" "dice_sh 8 bf16 16777216" "dice_sh 16 bf16 16777216" "dice_sh 2 bf16 16777216" "dice_sh 1 bf16 16777216"}; do
  set -- $cfg
  timeout -k 10 200 python -u tools/converge.py --env $1 --lanes 65536 --k $2 --precision $3 --replay $4 \
      --steps ${STEPS:-12000} --eval-every 250 --out $OUT > gpurun_out/converge_k_$1_$2_$3_$4.log 2>&1 || exit $?
done
echo ALLOK
