# k_solve: both tiles' rows loaded before either is consumed (sched_barrier): parity, then A/B
set -e -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shapes.py tests/test_gpu_parity.py tests/test_gpu_system.py > gpurun_out/r04_ssb_test.log 2>&1 || { tail -30 gpurun_out/r04_ssb_test.log; exit 1; }
tail -2 gpurun_out/r04_ssb_test.log
POPS="256" bash tools/ab_env.sh 3 'base=' 'var=' 2>&1 | tee gpurun_out/r04_ssb_ab.txt
for r in 1 2; do for v in base var; do
  TBLUP_GPU_LIB=ab/$v.so timeout -k 10 300 python bench.py --config config5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5_$v.log 2> gpurun_out/c5_$v.err
  python3 -c "import json;d=json.loads(open('gpurun_out/c5_$v.log').read().strip().splitlines()[-1]);print('config5', '$v', d['value'], d['kernel_ms_per_step'])" | tee -a gpurun_out/r04_ssb_ab.txt
done; done
