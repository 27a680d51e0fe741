# round 4: D-unit slicing forced (2 slices from column 1 / from column 4; 1 slice everywhere) vs the planner
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
POPS="256 128" bash tools/ab_env.sh 3 "var=" "d2=" "d2j4=" "d1=" 2>&1 | tee gpurun_out/r04_nds.txt
