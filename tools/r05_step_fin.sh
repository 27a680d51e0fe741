# final E-unit rule (var) vs the previous commit (base): parity suites, then pops 256 / 128
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS="tests/test_gpu_schedule.py tests/test_gpu_shapes.py tests/test_gpu_parity.py" POPS="256 128" ROUNDS=3 OUT=r05_fin bash tools/gpu_step.sh base= var= || exit 1
