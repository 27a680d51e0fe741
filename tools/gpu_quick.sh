# Quick GPU pass: the full -m gpu suite, the default bench line, and bench lines at smaller
# populations (pop 32 / 64 / 128: the per-GPU shares of config 3 and of a strong-scaled pop 256).
#   usage: bash tools/gpu_quick.sh TAG [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dev}
O=gpurun_out
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $O/gputest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/gputest_$TAG.log; tail -3 $O/gputest_$TAG.log; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$TAG.log 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 1; }
tail -1 $O/bench_$TAG.log | cut -c1-400
for p in 32 64 128; do
  timeout -k 10 200 python bench.py --pop $p --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pop${p}_$TAG.log 2> $O/bench_pop${p}_$TAG.err || { tail -20 $O/bench_pop${p}_$TAG.err; exit 1; }
  tail -1 $O/bench_pop${p}_$TAG.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($p, d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done
echo quick done
