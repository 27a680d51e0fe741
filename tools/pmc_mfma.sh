# MFMA utilisation counters for the bench kernels (one PMC pass; counters only, no tracing domains).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_mfma.log 2>&1 || { echo "pmc mfma failed"; tail -20 gpurun_out/pmc_mfma.log; exit 1; }
ls gpurun_out/pmc_mfma
