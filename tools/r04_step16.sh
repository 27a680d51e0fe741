# round 4: k_solve stages X_I into LDS under the tile stream -- solve GPU tests, A/B at config 2
# (pop 256) and config 5 (3 traits)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_gpu_schedule.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04_xs.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04_xs.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r04_xs.log | head -20; exit 1; }
POPS="256" bash tools/ab_env.sh 3 "base=" "var=" 2>&1 | tee gpurun_out/r04_xs_ab.txt || exit 1
for r in 1 2; do for v in base var; do
  TBLUP_GPU_LIB=ab/$v.so timeout -k 10 200 python bench.py --config config5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab5_$v.log 2> gpurun_out/ab5_$v.err || { tail -5 gpurun_out/ab5_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab5_$v.log').read().strip().splitlines()[-1]);print('config5', '$v', d['value'], d['kernel_ms_per_step'])" | tee -a gpurun_out/r04_xs_ab.txt
done; done
