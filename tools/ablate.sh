# Phase ablation: bench.py per TBLUP_DBG_SKIP value (results are wrong when set; timing only).
# Needs the diagnostic build: bash tools/ab_build_defs.sh 'diag=-DTBLUP_DIAG_BUILD' (TBLUP_GPU_LIB=ab/diag.so below);
# the production library ignores the ablation variables.
# usage: bash tools/ablate.sh "0 1024 2048 4096"
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in $1; do
  TBLUP_GPU_LIB=ab/diag.so TBLUP_DBG_SKIP=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abl_$v.log 2>&1 || { tail -5 gpurun_out/abl_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abl_$v.log').read().strip().splitlines()[-1]); print('skip', $v, d['value'], d['kernel_ms_per_step'])"
done
