# convergence band test (3 build seeds x {bf16, fp32} x 3 envs vs 5 reference seeds)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_converge_gpu.py -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/conv_tests.log 2>&1
echo CONV_RC=$?
