# E-unit policies: auto (every idle CU) vs only columns every tile of which gets one (TBLUP_DIAG_E=2)
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS=none POPS="128 64 96 32 160" ROUNDS=2 OUT=r05_epol bash tools/gpu_step.sh e0=TBLUP_DIAG_E=0 eauto= efull=TBLUP_DIAG_E=2 || exit 1
