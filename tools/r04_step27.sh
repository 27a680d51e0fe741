# LDS-DMA rings as inline asm (SYRK / GEMM1): schedule + shape parity, then interleaved A/B
set -e -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_shapes.py > gpurun_out/r04_asm_test.log 2>&1 || { tail -30 gpurun_out/r04_asm_test.log; exit 1; }
tail -2 gpurun_out/r04_asm_test.log
POPS="256 128" bash tools/ab_env.sh 2 'base=' 'none=' 'syrk=' 'gemm=' 'var=' 2>&1 | tee gpurun_out/r04_asm_ab.txt
