# round 4: non-temporal L-tile loads in the solves -- schedule/shape tests, A/B at pop 256 / 128
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_shapes.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r04_ntsolve.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04_ntsolve.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r04_ntsolve.log | head -20; exit 1; }
POPS="256 128 32" bash tools/ab_env.sh 3 "base=" "var=" 2>&1 | tee gpurun_out/r04_ntsolve_ab.txt
