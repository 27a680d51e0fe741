# A/B of two library builds with TBLUP_LAST_TERM=1 (the base build ignores it) at pop 32-256.
#   usage (on the GPU box): bash tools/ab_last_term.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lt_test.log 2>&1 || { tail -30 gpurun_out/lt_test.log; exit 1; }
tail -1 gpurun_out/lt_test.log
for rep in 1 2; do
for P in 32 64 128 192 256; do
  for v in base var; do
  TBLUP_LAST_TERM=1 TBLUP_GPU_LIB=ab/$v.so timeout -k 10 120 python bench.py --pop $P --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/lt.log 2> gpurun_out/lt.err || { tail -5 gpurun_out/lt.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/lt.log').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print($P, '$v', d['value'], k['chol_diag'], k['chol_offdiag'])"
  done
done
done
