# diagonal-target partials in up to three block slices, the planner counting the E-units' term (var)
# vs HEAD (base)
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS="tests/test_gpu_schedule.py tests/test_gpu_shapes.py" POPS="128 64 32 96 256" ROUNDS=2 OUT=r05_nds bash tools/gpu_step.sh base= var= || exit 1
timeout -k 10 200 python tools/wg_trace.py gpurun_out/wgt_nds128.npy --pop 128 > gpurun_out/wgt_nds128.txt 2>&1
