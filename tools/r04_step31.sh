# k_sys_tiles_st with 128-B stages (full lines, 2-deep ring): parity on that build, then A/B
set -e -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TBLUP_GPU_LIB=ab/sb128.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shapes.py tests/test_gpu_parity.py > gpurun_out/r04_sb128_test.log 2>&1 || { tail -30 gpurun_out/r04_sb128_test.log; exit 1; }
tail -2 gpurun_out/r04_sb128_test.log
POPS="256 128" bash tools/ab_env.sh 3 'base=' 'var=' 'sb128=' 2>&1 | tee gpurun_out/r04_sb128_ab.txt
