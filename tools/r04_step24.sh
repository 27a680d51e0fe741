# k_sys_tiles decomposition (diagnostic skip bits, timing only): full / no MFMA / no stores / neither
set -e
cd $GRAFT_REPO_ROOT
POPS=256 bash tools/ab_env.sh 2 'full=' 'nocomp=TBLUP_DBG_SKIP=262144' 'nostore=TBLUP_DBG_SKIP=196608' 'loadonly=TBLUP_DBG_SKIP=458752' 2>&1 | tee gpurun_out/r04_systiles_decomp.txt
