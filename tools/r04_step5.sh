# round 4: A/B of launches ahead at config 2 (compile-time masks), then last-term mode at pop 128
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
POPS="256" bash tools/ab_env.sh 2 "var=" "m8=" "m32=" "m40=" 2>&1 | tee gpurun_out/r04_ahead_mask.txt || exit 1
POPS="128" bash tools/ab_env.sh 2 "var=" "lt=TBLUP_LAST_TERM=1" 2>&1 | tee gpurun_out/r04_lastterm128.txt
