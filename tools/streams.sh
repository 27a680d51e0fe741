set -o pipefail
cd $GRAFT_REPO_ROOT
for n in ${NS:-1 2 3 4}; do
  TBLUP_STREAMS=$n timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $EXTRA > gpurun_out/streams_$n.log 2>&1 || { echo "streams $n failed"; tail -5 gpurun_out/streams_$n.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/streams_$n.log').read().strip().splitlines()[-1]); print('streams $n', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done
