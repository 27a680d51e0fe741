# A/B: the two SNP-form solve kernels (TBLUP_SOLVE_CHAIN=0 / 1) at pop 32-256 after the
# schedule and parity tests (results must be bit-identical; the checksum column shows it).
#   usage (on the GPU box): bash tools/ab_solve_chain.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/chain_test.log 2>&1 || { tail -30 gpurun_out/chain_test.log; exit 1; }
tail -2 gpurun_out/chain_test.log
for P in 32 64 128 192 256; do
for ch in 0 1; do
  TBLUP_SOLVE_CHAIN=$ch timeout -k 10 120 python bench.py --pop $P --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/chain_${P}_$ch.log 2> gpurun_out/chain_${P}_$ch.err || { tail -5 gpurun_out/chain_${P}_$ch.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/chain_${P}_$ch.log').read().strip().splitlines()[-1]); print($P, $ch, d['value'], d['kernel_ms_per_step']['solve'], d['fitness_checksum'])"
done
done
TBLUP_SOLVE_CHAIN=1 timeout -k 10 120 python tools/solve_trace.py --pop 32 > gpurun_out/strace32.txt 2>&1
