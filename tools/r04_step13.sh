# round 4: K-last accumulation in the off-diagonal units (counts loaded under the X staging) --
# parity / schedule / shape GPU tests, then A/B against HEAD at pop 256 / 128 / 32
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04_klast.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04_klast.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r04_klast.log | head -20; exit 1; }
POPS="256 128 32" bash tools/ab_env.sh 3 "base=" "var=" 2>&1 | tee gpurun_out/r04_klast_ab.txt
