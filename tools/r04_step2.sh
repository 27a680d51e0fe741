# round 4: the D-unit column bound sweep (DD_MAX_J as A/B builds) + the current tree at pop 256
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
POPS="128 96" bash tools/ab_env.sh 2 "var=" "off=TBLUP_DIAG_D=0" "j2=" "j4=" "j5=" 2>&1 | tee gpurun_out/r04_ddmaxj.txt || exit 1
POPS="256" bash tools/ab_env.sh 2 "var=" 2>&1 | tee -a gpurun_out/r04_ddmaxj.txt
