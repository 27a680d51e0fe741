# scalars formed at the head of the persistent system-tile kernel's runs (var) vs the fused scalar +
# K_JJ launch after it (HEAD, base)
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS="tests/test_gpu_schedule.py tests/test_gpu_shapes.py tests/test_gpu_parity.py" POPS="128 256" ROUNDS=3 OUT=r05_sth bash tools/gpu_step.sh base= var= || exit 1
