# Phase ablation of the Cholesky kernels (timing only; results are wrong for masks != 0).
set -o pipefail
cd $GRAFT_REPO_ROOT
for m in ${MASKS:-0 1 2 4 8 16 32 64 128 256 512}; do
  TBLUP_DBG_SKIP=$m timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abl_$m.log 2>&1 || { echo "mask $m failed"; tail -5 gpurun_out/abl_$m.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abl_$m.log').read().strip().splitlines()[-1]); print('mask $m', d['kernel_ms_per_step'])"
done
