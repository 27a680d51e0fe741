set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS="tests/test_gpu_schedule.py tests/test_gpu_shapes.py" POPS="128 96 160" ROUNDS=3 OUT=r05_ltm bash tools/gpu_step.sh base= var= || exit 1
POPS="256 192" bash tools/ab_env.sh 2 'auto=' 'chain1=TBLUP_SOLVE_CHAIN=1' 2>&1 | tee gpurun_out/r05_chain256.txt
