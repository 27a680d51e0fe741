set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_evolver.py tests/test_main_flow.py tests/test_gpu_shards.py tests/test_keystore.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/r06b_test.log 2>&1 || { tail -30 $O/r06b_test.log; exit 1; }
tail -2 $O/r06b_test.log
timeout -k 10 300 python tools/generation_bench.py 16 1024 > $O/r06b_gen1024.log 2>&1 || { tail -20 $O/r06b_gen1024.log; exit 1; }
timeout -k 10 300 python tools/generation_bench.py 24 256 > $O/r06b_gen256.log 2>&1 || { tail -20 $O/r06b_gen256.log; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29604 tools/generation_bench.py 16 1024 > $O/r06b_gen1024_w4.log 2>&1 || { tail -30 $O/r06b_gen1024_w4.log; exit 1; }
for f in $O/r06b_gen1024.log $O/r06b_gen256.log $O/r06b_gen1024_w4.log; do
python3 - $f <<'PY'
import json, statistics as s, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); a=d['gpu_generation_ms_all'][1:]
        seg=d['evolve_segments_last_gen_ms']
        print(d['pop'], d['world'], 'best', min(a), 'median', round(s.median(a),2), {k: seg[k] for k in ('ev_candidates','ev_arrays','ev_bind_record','ev_rows_landed','ev_compact','ev_gather')})
PY
done
