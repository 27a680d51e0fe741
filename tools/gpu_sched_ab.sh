# Schedule A/B: correctness of the Cholesky schedules, then bench lines per (population, schedule).
#   usage: bash tools/gpu_sched_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dev}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/gputest_sched_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gputest_sched_$TAG.log; tail -3 $O/gputest_sched_$TAG.log; [ $rc -eq 0 ] || exit 1
run() {  # name pop env...
  local name=$1 pop=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --pop $pop --steps 20 --warmup 5 --no-cpu-baseline > $O/ab_${name}_$TAG.log 2> $O/ab_${name}_$TAG.err || { tail -20 $O/ab_${name}_$TAG.err; exit 1; }
  tail -1 $O/ab_${name}_$TAG.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['fitness_checksum'])"
}
for pop in 256 128 64 32; do
  run p${pop}_classic $pop TBLUP_AHEAD=0
  run p${pop}_q $pop TBLUP_AHEAD=0
  run p${pop}_ahead_q $pop TBLUP_AHEAD=1
done
run p256_ahead_q_nrs2 256 TBLUP_AHEAD=1 TBLUP_NRS=2
run p32_ahead_q_nrs2 32 TBLUP_AHEAD=1 TBLUP_NRS=2
echo ab done
