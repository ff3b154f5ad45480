set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bnr or bn_reduce or bn_backward_reduce" > gpurun_out/bnr_inner_tests.log 2>&1 && tail -3 gpurun_out/bnr_inner_tests.log && AB_VAR=DDL_FUSE_BN_REDUCE_INNER AB_VALUES="1 0" ROUNDS=2 bash scripts/gpu_r3_ab.sh
