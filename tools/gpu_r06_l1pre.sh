#!/bin/bash
# round 6: the target critic's layer 1 over s' formed under the policy's fc2 stream (library
# tools/_abh/librlmd_amd_l1prenew.so) — learn / target-pairing / full-size / smoke-matrix tests on it,
# then same-box traces (new / the tree's library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NEW=tools/_abh/librlmd_amd_l1prenew.so
RLMD_LIB_PATH=$NEW timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_learn_gpu.py tests/test_target_pair_gpu.py tests/test_fullsize_gpu.py tests/test_smoke_matrix_gpu.py \
  > gpurun_out/r06_l1pre_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_l1pre_tests.log; [ $rc -eq 0 ] || exit $rc
RLMD_LIB_PATH=$NEW timeout -k 10 120 python -u tools/probe/params_after_steps.py gpurun_out/l1pre_new.npz || exit 1
timeout -k 10 120 python -u tools/probe/params_after_steps.py gpurun_out/l1pre_old.npz || exit 1
python -c "
import numpy as np
a, b = np.load('gpurun_out/l1pre_new.npz'), np.load('gpurun_out/l1pre_old.npz')
for k in a.files: print(k, 'bit-equal' if np.array_equal(a[k], b[k], equal_nan=True) else 'DIFFERENT')
"
timeout -k 10 700 bash tools/gpu_trace_ab.sh l1pre "c2:RLMD_LIB_PATH=$NEW c2:- c3:RLMD_LIB_PATH=$NEW c3:- c2:RLMD_LIB_PATH=$NEW c2:-" \
  > gpurun_out/r06_l1pre_ab.log 2>&1 || { tail -20 gpurun_out/r06_l1pre_ab.log; exit 1; }
grep -E "==|fwd_rows|qeval|critic_update|actor_update" gpurun_out/tab_l1pre/summary.txt
