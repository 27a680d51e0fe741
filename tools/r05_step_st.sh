# per-individual scalars: wave-shuffle sums, the u / rhs rows after the K_JJ epilogue (var) vs HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS="tests/test_gpu_schedule.py tests/test_gpu_shapes.py tests/test_gpu_parity.py" POPS="128 256" ROUNDS=2 OUT=r05_st bash tools/gpu_step.sh base= var= || exit 1
