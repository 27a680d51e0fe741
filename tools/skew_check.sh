# Skewed two-group column schedule A/B: parity tests and bench with TBLUP_SKEW=1, then the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
TBLUP_SKEW=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gsk.log 2>&1
rc=$?; tail -3 gpurun_out/gsk.log; [ $rc -eq 0 ] || exit 1
TBLUP_SKEW=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bsk.log 2>&1 || { tail -5 gpurun_out/bsk.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bsk.log').read().strip().splitlines()[-1]); print('skew', d['value'], d['kernel_ms_per_step'])"
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bref.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bref.log').read().strip().splitlines()[-1]); print('ref', d['value'], d['kernel_ms_per_step'])"
