# round 4: launches ahead at pop 256 by compile-time mask (bit j: launch j computes column j+1's
# partial sums), then the D-units-beside-the-diagonal bound at pop 96 / 128
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
POPS="256" bash tools/ab_env.sh 3 "var=" "m32=" "m48=" "m16=" "m56=" 2>&1 | tee gpurun_out/r04_ahead_mask.txt || exit 1
POPS="96 128" bash tools/ab_env.sh 2 "off=TBLUP_DIAG_D=0" "j2=" "var=" "j4=" 2>&1 | tee gpurun_out/r04_ddmaxj.txt
