# E-units (TBLUP_DIAG_E) and the scalars fused into the K_JJ epilogue launch: parity, then A/B
# against HEAD's library (ab/base.so) and E-units off, then a workgroup trace at pop 128
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTS=all POPS="128 256 64" ROUNDS=2 OUT=r05_eunits bash tools/gpu_step.sh base= e0=TBLUP_DIAG_E=0 eauto= || exit 1
timeout -k 10 200 python tools/wg_trace.py gpurun_out/wgt_e128.npy --pop 128 > gpurun_out/wgt_e128.txt 2>&1
