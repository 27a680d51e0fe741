# A/B of two library builds (tools/ab_build.sh: ab/base.so = HEAD, ab/var.so = working tree) at
# pop 32-256 after the schedule tests.   usage (on the GPU box): bash tools/ab_offdiag_plan.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_schedule.py -x -q --timeout 200 --timeout-method thread > gpurun_out/nds_test.log 2>&1 || { tail -30 gpurun_out/nds_test.log; exit 1; }
tail -1 gpurun_out/nds_test.log
for rep in 1 2; do
for P in 32 64 128 192 256; do
  for v in base var; do
  TBLUP_GPU_LIB=ab/$v.so timeout -k 10 120 python bench.py --pop $P --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/nds.log 2> gpurun_out/nds.err || { tail -5 gpurun_out/nds.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/nds.log').read().strip().splitlines()[-1]); print($P, '$v', d['value'], d['kernel_ms_per_step']['chol_offdiag'])"
  done
done
done
