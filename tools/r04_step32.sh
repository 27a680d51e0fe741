# schedule policies re-measured after the rings stopped draining (runtime knobs, one build)
set -e -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
POPS="128 256" bash tools/ab_env.sh 2 'auto=' 'ahead1=TBLUP_AHEAD=1' 'ahead0=TBLUP_AHEAD=0' 'lt1=TBLUP_LAST_TERM=1' 'nrs2=TBLUP_NRS=2' 2>&1 | tee gpurun_out/r04_policy_ab.txt
