# round 4: the w accumulation over the traits present only -- full GPU suite, A/B at pop 256 /
# 128 and config 5
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04_wtr.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04_wtr.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r04_wtr.log | head -20; exit 1; }
POPS="256 128" bash tools/ab_env.sh 3 "base=" "var=" 2>&1 | tee gpurun_out/r04_wtr_ab.txt || exit 1
for r in 1 2; do for v in base var; do
  TBLUP_GPU_LIB=ab/$v.so timeout -k 10 200 python bench.py --config config5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab5_$v.log 2> gpurun_out/ab5_$v.err || { tail -5 gpurun_out/ab5_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab5_$v.log').read().strip().splitlines()[-1]);print('config5', '$v', d['value'], d['kernel_ms_per_step'])" | tee -a gpurun_out/r04_wtr_ab.txt
done; done
