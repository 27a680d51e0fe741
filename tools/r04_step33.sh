# T-units: GEMM1's first A stage issued before the count wait (inline asm): parity, then A/B
set -e -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_shapes.py tests/test_gpu_parity.py > gpurun_out/r04_early_test.log 2>&1 || { tail -30 gpurun_out/r04_early_test.log; exit 1; }
tail -2 gpurun_out/r04_early_test.log
POPS="256 128" bash tools/ab_env.sh 3 'base=' 'var=' 2>&1 | tee gpurun_out/r04_early_ab.txt
