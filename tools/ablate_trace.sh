# Per-kernel average durations under phase-ablation masks (timing only; results are wrong for masks != 0).
# Needs the diagnostic build: bash tools/ab_build_defs.sh 'diag=-DTBLUP_DIAG_BUILD' (TBLUP_GPU_LIB=ab/diag.so below);
# the production library ignores the ablation variables.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in ${MASKS:-0 4 8 16 256 512}; do
  TBLUP_GPU_LIB=ab/diag.so TBLUP_DBG_SKIP=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abl_$m -o t --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abl_$m.log 2>&1 || { echo "mask $m failed"; tail -5 gpurun_out/abl_$m.log; exit 1; }
  python3 - "$m" <<'PY'
import csv, sys
m = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/abl_{m}/t_kernel_stats.csv")))
out = []
for r in rows:
    name = r["Name"].split("(")[0].replace("tblup::", "").replace("void ", "").split("<")[0]
    if name.startswith("k_"):
        out.append(f"{name}={float(r['AverageNs'])/1e3:.1f}us")
print("mask", m, " ".join(sorted(out)))
PY
done
