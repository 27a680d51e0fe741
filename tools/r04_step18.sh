# round 4: chained solve in individual-major grid order -- chain GPU tests, solve timeline at pop 128,
# A/B against HEAD (level-major) at pop 32 / 64 / 128
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_schedule.py tests/test_gpu_shards.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r04_imaj.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04_imaj.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r04_imaj.log | head -20; exit 1; }
timeout -k 10 120 python tools/solve_trace.py --pop 128 > gpurun_out/solve_trace_r04c.txt 2>&1; tail -12 gpurun_out/solve_trace_r04c.txt
POPS="32 64 128" bash tools/ab_env.sh 3 "base=" "var=" 2>&1 | tee gpurun_out/r04_imaj_ab.txt
