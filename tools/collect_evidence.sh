# Copy one evidence run's summaries (tools/gpu_evidence.sh TAG, merged into gpurun_out/) into
# profiles/ under that tag, and make its PMC summaries the bench's defaults.   usage: bash tools/collect_evidence.sh r03a
set -e
T=$1; O=gpurun_out; P=profiles
tail -1 $O/bench_$T.log > $P/${T}_bench.jsonl
for c in config3 config4 config5 pop32 pop64 pop128; do
  [ -f $O/bench_${c}_$T.log ] && tail -1 $O/bench_${c}_$T.log > $P/${T}_bench_$c.jsonl
done
cp $O/prof_$T/trace_kernel_stats.csv $P/${T}_kernel_stats.csv
# the bench's rocprof-timed roofline reads profiles/kernel_stats.csv only for the workload its
# sidecar names (tools/gpu_evidence.sh profiles the default bench: config 2, pop 256 on one GPU)
cp $O/prof_$T/trace_kernel_stats.csv $P/kernel_stats.csv
echo '{"config": "config2", "pop_per_gpu": 256, "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline", "source": "'$T'"}' > $P/kernel_stats.meta.json
cp $O/prof_$T/trace_domain_stats.csv $P/${T}_domain_stats.csv
cp $O/prof_$T/trace_kernel_trace.csv $P/${T}_kernel_trace.csv
cp $(find $O/pmcf_$T -name "*counter_collection.csv" | head -1) $P/${T}_pmc_fetch.csv
cp $(find $O/pmcw_$T -name "*counter_collection.csv" | head -1) $P/${T}_pmc_write.csv
cp $(find $O/pmcm_$T -name "*counter_collection.csv" | head -1) $P/${T}_pmc_mfma.csv
cp $(find $O/pmcs_$T -name "*counter_collection.csv" | head -1) $P/${T}_pmc_stall.csv
cp $O/pmc_traffic_$T.json $P/pmc_traffic.json
cp $O/pmc_mfma_$T.json $P/pmc_mfma.json
tail -1 $O/generation_$T.log > $P/${T}_generation.json
for f in $O/generation_w*_$T.log; do [ -f $f ] && grep '^{' $f | tail -1; done > $P/${T}_generation_ranks.jsonl
grep config $O/intracv_$T.log > $P/${T}_intracv.jsonl
[ -f $O/knockout_$T.log ] && tail -1 $O/knockout_$T.log > $P/${T}_knockout.json
cp $O/wg_trace_$T.txt $P/${T}_wg_trace.txt
cp $O/wg_trace128_$T.txt $P/${T}_wg_trace_pop128.txt
cp $O/mfma_peak_$T.json $P/${T}_mfma_peak.json
cp $O/fp4_probe_$T.json $P/${T}_fp4_probe.json
cp $O/gputest_$T.log $P/${T}_gputest.log 2>/dev/null || true
ls -la $P | grep $T
