# persistent super-tile system tiles (k_sys_tiles_st): parity first, then interleaved A/B
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_shapes.py -k "persistent" 2>&1 | tail -8
POPS="256 128 64 32" bash tools/ab_env.sh 2 'base=' 'off=TBLUP_SYS_ST=0' 'st=TBLUP_SYS_ST=1' 2>&1 | tee gpurun_out/r04_sysst_ab.txt
