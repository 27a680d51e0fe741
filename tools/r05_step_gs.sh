# k_sys_tiles_st unit mapping: each XCD a contiguous eighth of the units, groups of SYS_GS workgroups
# walking one share interleaved (var: 2; gs1 / gs4) vs HEAD (base)
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS="tests/test_gpu_shapes.py tests/test_gpu_parity.py" POPS="256 128" ROUNDS=2 OUT=r05_gs bash tools/gpu_step.sh base= gs1= var= gs4= || exit 1
