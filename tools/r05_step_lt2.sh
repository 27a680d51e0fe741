# last-term mask with the E-units: diagonal 7's last SYRK term from off-diagonal launch 6 (bit 7),
# whose T-units the E-units have shortened
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS=none POPS="128 96 160" ROUNDS=2 OUT=r05_lt2 bash tools/gpu_step.sh auto= lt8a=TBLUP_LT_MASK=0x8A lt82=TBLUP_LT_MASK=0x82 || exit 1
