#!/bin/bash
# Kernel-trace + FETCH_SIZE / WRITE_SIZE profiles of the config-4 (4 MiB chunks) and mixed-size
# (config-5 size classes, device-resident) verify launches, summarised into
# gpurun_out/prof_<tag>/summary.{txt,json} for bench.py's roofline `traffic`.
# shard4m is profiled on one 64 GiB pass: the same per-launch shape as each of the default run's
# four passes (16384 x 4 MiB).  mixed: rank 0's 674 chunks, 8,620,183,509 bytes per launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
prof() {  # tag kernel alg_bytes description workload [bench args]
  local tag=$1 kern=$2 alg=$3 desc=$4 w=$5; shift 5
  bash scripts/profile.sh $w $tag "$@" > gpurun_out/prof_$tag.log 2>&1 || { echo PROF_${tag}_FAIL; exit 1; }
  python3 scripts/summarize_kernels.py gpurun_out/prof_$tag --json $kern $alg "$desc" gpurun_out/prof_$tag/summary.json \
    > /dev/null || exit 1
}
prof shard4m seg_crc_kernel 68719476736 "bench.py --workload shard4m --total-gib 64: one 64 GiB pass of 16384 x 4 MiB chunks (BASELINE config 4 per-launch shape)" shard4m --total-gib 64 --pass-gib 64
prof mixed seg_crc_kernel 8620183509 "bench.py --workload mixed: 674 chunks of 64 KiB-64 MiB, 10% ragged, packed unaligned, 8.03 GiB per launch" mixed
echo PROF_EXTRA_OK
