# three-launch DE step for pop > CU count: GPU evolver tests, then the pop-1024 / 256 generation
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_evolver.py tests/test_gpu_system.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_gen2_test.log 2>&1; rc=$?; tail -2 gpurun_out/r05_gen2_test.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/generation_bench.py 16 1024 > gpurun_out/gen_w1_1024_r05k.log 2>&1 || { tail -5 gpurun_out/gen_w1_1024_r05k.log; exit 1; }
timeout -k 10 300 python tools/generation_bench.py 24 > gpurun_out/gen_w1_256_r05k.log 2>&1 || { tail -5 gpurun_out/gen_w1_256_r05k.log; exit 1; }
for f in gen_w1_1024_r05k gen_w1_256_r05k; do python3 -c "
import json, statistics as s
d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); a=d['gpu_generation_ms_all'][1:]
print('$f', 'best', min(a), 'median', round(s.median(a),2), 'max', max(a), d['evolve_segments_last_gen_ms'])"; done
