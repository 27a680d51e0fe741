# round 4: GEMM1's first stage issued ahead of the unit prologue -- full GPU suite, A/B at pop 256 /
# 128, and the workgroup trace with the T-units' phase stamps
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04_g1pre.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04_g1pre.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r04_g1pre.log | head -20; exit 1; }
POPS="256 128" bash tools/ab_env.sh 3 "base=" "var=" 2>&1 | tee gpurun_out/r04_g1pre_ab.txt || exit 1
timeout -k 10 200 python tools/wg_trace.py gpurun_out/wg_trace_ph.npy > gpurun_out/wg_trace_ph.txt 2>&1; grep -A9 "T-unit phases" gpurun_out/wg_trace_ph.txt
timeout -k 10 200 python tools/wg_trace.py gpurun_out/wg_trace_ph128.npy --pop 128 > gpurun_out/wg_trace_ph128.txt 2>&1; grep -A9 "T-unit phases" gpurun_out/wg_trace_ph128.txt
