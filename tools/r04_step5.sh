# round 4: A/B at config 2 -- column 0 inside the diagonal launch (auto at pop 256) vs its own launch,
# launches ahead (compile-time masks) -- then last-term mode at pop 128
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
POPS="256" bash tools/ab_env.sh 2 "var=" "nofuse=TBLUP_FUSE_COL0=0" "m8=" "m32=" "m40=" 2>&1 | tee gpurun_out/r04_ahead_mask.txt || exit 1
POPS="128" bash tools/ab_env.sh 2 "var=" "lt=TBLUP_LAST_TERM=1" "fuse=TBLUP_FUSE_COL0=1" 2>&1 | tee gpurun_out/r04_lastterm128.txt
