# k_sys_tiles_st: parity, then its decomposition (skip bits) and ring depth 4 vs 3
set -e -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_shapes.py -k "persistent" > gpurun_out/r04_sysst_test.log 2>&1 || { tail -30 gpurun_out/r04_sysst_test.log; exit 1; }
tail -3 gpurun_out/r04_sysst_test.log
POPS="256" bash tools/ab_env.sh 2 'base=' 'var=' 'd4=' 'nocomp=TBLUP_DBG_SKIP=262144' 'nostore=TBLUP_DBG_SKIP=196608' 'loadonly=TBLUP_DBG_SKIP=458752' 2>&1 | tee gpurun_out/r04_sysst_decomp.txt
