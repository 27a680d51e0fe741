# round 4: the D-units-beside-the-diagonal bound (DD_MAX_J, compile-time A/B builds) at pop 96 / 128
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
POPS="96 128" bash tools/ab_env.sh 3 "off=TBLUP_DIAG_D=0" "j2=" "var=" "j4=" 2>&1 | tee gpurun_out/r04_ddmaxj.txt
