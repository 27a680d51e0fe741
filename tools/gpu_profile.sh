# Round profiling: kernel trace + stats, then one PMC pass per counter (never combined with tracing domains).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gputest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gputest.log
tail -3 gpurun_out/gputest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.log 2>&1 || { echo "kernel-trace failed"; tail -20 gpurun_out/prof_bench_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_$TAG.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/pmc_write_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG -type f | head -20
