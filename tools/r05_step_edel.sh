# E-units with partial columns as the automatic rule (var); their start delayed 8 / 13 us (A/B builds)
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS=none POPS="128 96 160" ROUNDS=2 OUT=r05_edel bash tools/gpu_step.sh var= d800= d1300= || exit 1
