# hipGraph replay probe (a Python exception there does not stop the run; a fault, abort or
# time limit does), then the round evidence.   usage: bash tools/probe_then_evidence.sh r02f
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dev}
timeout -k 10 180 python -u tools/graph_probe.py 40 > gpurun_out/graph_probe_$TAG.log 2>&1
rc=$?; echo "graph probe rc=$rc"; tail -2 gpurun_out/graph_probe_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
bash tools/gpu_evidence.sh $TAG
