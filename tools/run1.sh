set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputest1.log 2>&1 || { tail -30 gpurun_out/gputest1.log; exit 1; }
tail -2 gpurun_out/gputest1.log
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench1.log 2>&1 || { tail -5 gpurun_out/bench1.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench1.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'])"
bash tools/phase_trace.sh "0"
