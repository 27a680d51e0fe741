# last-term mask sweep at pop 128 with the E-units (bit J: diagonal J's last term from launch J-1)
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS=none POPS="128" ROUNDS=2 OUT=r05_lt3 bash tools/gpu_step.sh auto= m0e=TBLUP_LT_MASK=0x0E m1a=TBLUP_LT_MASK=0x1A m2a=TBLUP_LT_MASK=0x2A m4a=TBLUP_LT_MASK=0x4A m08=TBLUP_LT_MASK=0x08 m02=TBLUP_LT_MASK=0x02 m3e=TBLUP_LT_MASK=0x3E || exit 1
