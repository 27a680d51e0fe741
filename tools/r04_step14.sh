# round 4: batched FP4 system tiles + int16 counts (default) vs in-tile int8 system tiles (A/B build)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
POPS="256 128" bash tools/ab_env.sh 2 "var=" "nost=" 2>&1 | tee gpurun_out/r04_nost.txt
