set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gputest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gputest.log
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --profile-json gpurun_out/prof_r01.json > gpurun_out/bench.log 2> gpurun_out/bench.err && tail -2 gpurun_out/bench.log
