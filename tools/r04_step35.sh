# persistent vs per-tile system tiles now that the per-tile ring keeps its prefetch (runtime knob)
set -e -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
POPS="256 128 64" bash tools/ab_env.sh 2 'auto=' 'tile=TBLUP_SYS_ST=0' 'st=TBLUP_SYS_ST=1' 2>&1 | tee gpurun_out/r04_sysst2_ab.txt
