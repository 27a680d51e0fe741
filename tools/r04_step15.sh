# round 4: SYRK blocks by row pairs (fewer A-fragment LDS reads in the D-units and the diagonal's
# phase A) -- full GPU suite, then A/B against HEAD at pop 256 / 128
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04_syrk.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04_syrk.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputest_r04_syrk.log | head -20; exit 1; }
POPS="256 128" bash tools/ab_env.sh 3 "base=" "var=" 2>&1 | tee gpurun_out/r04_syrk_ab.txt
