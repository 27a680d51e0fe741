# launches ahead by mask at pop 128 now that the E-units run beside the diagonal launches
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS=none POPS="128" ROUNDS=2 OUT=r05_am bash tools/gpu_step.sh var= am10= am08= am18= am04= || exit 1
