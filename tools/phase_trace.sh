# Per-launch durations of one pipeline step under phase-ablation masks (timing only; results
# Needs the diagnostic build: bash tools/ab_build_defs.sh 'diag=-DTBLUP_DIAG_BUILD' (TBLUP_GPU_LIB=ab/diag.so below);
# the production library ignores the ablation variables.
# are wrong for masks != 0).  usage: bash tools/phase_trace.sh "0 32 64 128"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in $1; do
  TBLUP_GPU_LIB=ab/diag.so TBLUP_DBG_SKIP=$m timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ph_$m -o t --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ph_$m.log 2>&1 || { echo "mask $m failed"; tail -5 gpurun_out/ph_$m.log; exit 1; }
  echo "== mask $m"
  python3 tools/trace_summary.py gpurun_out/ph_$m/t_kernel_trace.csv > gpurun_out/ph_$m.txt && cat gpurun_out/ph_$m.txt
done
