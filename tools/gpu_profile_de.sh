# DE step profile: kernel trace/stats of tools/de_bench.py, then FETCH_SIZE and WRITE_SIZE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_de_$TAG -o trace --output-format csv -- python3 tools/de_bench.py > gpurun_out/prof_de_$TAG.log 2>&1 || { echo "kernel-trace failed"; tail -20 gpurun_out/prof_de_$TAG.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_de_fetch_$TAG -o pmc --output-format csv -- python3 tools/de_bench.py > gpurun_out/pmc_de_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_de_fetch_$TAG.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_de_write_$TAG -o pmc --output-format csv -- python3 tools/de_bench.py > gpurun_out/pmc_de_write_$TAG.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/pmc_de_write_$TAG.log; exit 1; }
find gpurun_out/prof_de_$TAG gpurun_out/pmc_de_fetch_$TAG gpurun_out/pmc_de_write_$TAG -type f
