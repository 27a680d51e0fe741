# T-units of tiles their E-units started dispatched last, and partial E-unit columns (TBLUP_DIAG_E=3)
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS="tests/test_gpu_schedule.py tests/test_gpu_shapes.py" POPS="128 96 160 64" ROUNDS=2 OUT=r05_eord bash tools/gpu_step.sh base= var= e3=TBLUP_DIAG_E=3 || exit 1
