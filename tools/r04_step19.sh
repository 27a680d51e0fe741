# round 4: the prediction from the 2-bit packed split rows -- full GPU suite, A/B at pop 256 / 128 / 32
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04_pk.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04_pk.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r04_pk.log | head -20; exit 1; }
POPS="256 128 32" bash tools/ab_env.sh 3 "base=" "var=" 2>&1 | tee gpurun_out/r04_pk_ab.txt
