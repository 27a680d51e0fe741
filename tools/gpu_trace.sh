# Quick per-dispatch kernel trace of a short bench run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dev}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$TAG -o t --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/trace_$TAG.log 2>&1 || { tail -20 gpurun_out/trace_$TAG.log; exit 1; }
grep '"value"' gpurun_out/trace_$TAG.log | cut -c1-300
