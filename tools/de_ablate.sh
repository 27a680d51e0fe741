# DE step phase ablation (TBLUP_DE_DBG: 1 no jump correlation, 2 no mask recurrence, 4 no stream)
# Needs the diagnostic build: bash tools/ab_build_defs.sh 'diag=-DTBLUP_DIAG_BUILD' (TBLUP_GPU_LIB=ab/diag.so below);
# the production library ignores the ablation variables.
cd $GRAFT_REPO_ROOT
for v in 0 1 2 4 3 7; do
  echo "dbg=$v"
  TBLUP_GPU_LIB=ab/diag.so TBLUP_DE_DBG=$v timeout -k 10 60 python tools/de_bench.py > gpurun_out/de_abl_$v.log 2>&1 || { tail -5 gpurun_out/de_abl_$v.log; exit 1; }
  cut -c1-140 gpurun_out/de_abl_$v.log
done
