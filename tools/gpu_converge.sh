# Convergence sweep on the GPU box: coin / dice / dice_sh INSURED, SAC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/converge_${TAG:-x}.jsonl
rm -f $OUT
for cfg in ${CFGS:-"coin 65536 8 bf16" "dice 65536 8 bf16" "dice_sh 65536 8 bf16"}; do
  set -- ${cfg//:/ }
  timeout -k 10 ${TLIM:-240} python -u tools/converge.py --env $1 --lanes $2 --k $3 --precision $4 \
      --steps ${STEPS:-20000} --eval-every ${EVERY:-1000} --out $OUT ${EXTRA} > gpurun_out/converge_${TAG:-x}_$1_$2_$3_$4.log 2>&1 || exit $?
done
echo CONVERGE_DONE
