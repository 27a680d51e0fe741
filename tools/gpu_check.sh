# GPU check: full -m gpu suite, bench line, rocprof kernel trace/stats of the bench, e2e generation timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dev}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$TAG.log; tail -3 gpurun_out/gputest_$TAG.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.log 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.log 2>&1 || { echo "kernel-trace failed"; tail -20 gpurun_out/prof_bench_$TAG.log; exit 1; }
timeout -k 10 200 python tools/generation_bench.py > gpurun_out/generation_$TAG.log 2>&1 || { tail -20 gpurun_out/generation_$TAG.log; exit 1; }
cat gpurun_out/generation_$TAG.log
