# round 4: block-row chained solve -- chain / shape / schedule GPU tests, solve timeline at pop 128,
# then A/B against HEAD's tile-unit chain (pop 32 / 64 / 128; pop 256 with the chain forced on)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_schedule.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest_r04_chain.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04_chain.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r04_chain.log | head -20; exit 1; }
timeout -k 10 120 python tools/solve_trace.py --pop 128 > gpurun_out/solve_trace_r04.txt 2>&1; tail -12 gpurun_out/solve_trace_r04.txt
POPS="32 64 128" bash tools/ab_env.sh 3 "base=" "var=" 2>&1 | tee gpurun_out/r04_chain_ab.txt || exit 1
POPS="256" bash tools/ab_env.sh 2 "base=TBLUP_SOLVE_CHAIN=1" "var=TBLUP_SOLVE_CHAIN=1" "var0=TBLUP_SOLVE_CHAIN=0" 2>&1 | tee -a gpurun_out/r04_chain_ab.txt
