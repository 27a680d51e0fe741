# DE step: one launch (TBLUP_DE_SPLIT=100000) vs three (TBLUP_DE_SPLIT=1) at every population size
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do for v in 100000 1; do for P in 32 64 128 256 384 512 1024; do
  TBLUP_DE_SPLIT=$v timeout -k 10 200 python -c "import sys; sys.path.insert(0, 'tools'); import de_bench; de_bench.main(pop=$P, reps=30)" > gpurun_out/de_$v.log 2>&1 || { tail -5 gpurun_out/de_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/de_$v.log').read().strip().splitlines()[-1]); print('split>=$v', $P, round(d['gpu_de_ms_median'],4), round(d['gpu_de_ms_min'],4))" | tee -a gpurun_out/r05_de3_ab.txt
done; done; done
