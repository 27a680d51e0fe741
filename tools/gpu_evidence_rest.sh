# The tail of tools/gpu_evidence.sh (from the workgroup timelines on), for a run that stopped there.
#   usage: bash tools/gpu_evidence_rest.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export TAG=${1:-dev} O=gpurun_out
sed -n '/tools\/wg_trace.py \$O\/wg_trace_\$TAG.npy/,$p' tools/gpu_evidence.sh > /tmp/ev_rest.sh
bash -o pipefail /tmp/ev_rest.sh
