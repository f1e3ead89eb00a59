#!/bin/bash
# Copies what scripts/final_refresh.sh left under gpurun_out/ into profiles/ as <tag>_*.
# usage: scripts/collect_refresh.sh <tag>   (e.g. r02)
set -e
T=$1; O=gpurun_out; P=profiles
tail -1 $O/bench.log > $P/${T}_bench_default.jsonl
for w in update updio hostfed shard4m mixed sync; do tail -1 $O/bench_$w.log > $P/${T}_bench_$w.jsonl; done
cp $O/pytest_gpu.log $P/${T}_pytest_gpu.log
cp $O/smoke.log $P/${T}_smoke.log
cp $O/prof_headline/summary.json $P/${T}_pmc_summary.json
cp $O/prof_small4k/summary.json $P/${T}_small4k_pmc_summary.json
cp $O/prof_upd/summary.json $P/${T}_update_pmc_summary.json
cp $O/prof_updio/summary.json $P/${T}_updio_pmc_summary.json
for t in headline small4k upd updio; do
  n=$t; [ $t = upd ] && n=update
  cp $O/prof_$t/summary.txt $P/${T}_${n}_kernels_pmc.txt
  cp $O/prof_$t/kt/kt_kernel_stats.csv $P/${T}_${n}_rocprof_kernel_stats.csv
done
