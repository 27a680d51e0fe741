# DE step: wave-ballot crossover mask (var) vs the per-lane LDS atomics (ab/old.so); then the fused
# scalars' hoisted centring-sum gather (var) vs HEAD (base)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do for v in old var; do for P in 256 1024; do
  TBLUP_GPU_LIB=ab/$v.so timeout -k 10 200 python -c "import sys; sys.path.insert(0, 'tools'); import de_bench; de_bench.main(pop=$P, reps=30)" > gpurun_out/de_$v.log 2>&1 || { tail -5 gpurun_out/de_$v.log; exit 1; }
  echo "$v $P $(tail -1 gpurun_out/de_$v.log)" | tee -a gpurun_out/r05_de_ab.txt
done; done; done
TESTS=none POPS="128 256" ROUNDS=2 OUT=r05_hoist bash tools/gpu_step.sh base= var= || exit 1
