# DE step: three launches from pop 384 (var) vs one (base): bit-exact tests, then de_bench at 256 / 512 / 1024
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_evolver.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_de2_test.log 2>&1; rc=$?; tail -2 gpurun_out/r05_de2_test.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r05_de2_test.log | head; exit 1; }
for r in 1 2; do for v in base var; do for P in 256 512 1024; do
  TBLUP_GPU_LIB=ab/$v.so timeout -k 10 200 python -c "import sys; sys.path.insert(0, 'tools'); import de_bench; de_bench.main(pop=$P, reps=30)" > gpurun_out/de_$v.log 2>&1 || { tail -5 gpurun_out/de_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/de_$v.log').read().strip().splitlines()[-1]); print('$v', $P, round(d['gpu_de_ms_median'],4), round(d['gpu_de_ms_min'],4))" | tee -a gpurun_out/r05_de2_ab.txt
done; done; done
