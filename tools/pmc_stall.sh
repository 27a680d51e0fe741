# Wave-state breakdown (one PMC pass of SQ counters; counters only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d gpurun_out/pmc_stall -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_stall.log 2>&1 || { echo "pmc stall failed"; tail -20 gpurun_out/pmc_stall.log; exit 1; }
ls gpurun_out/pmc_stall
