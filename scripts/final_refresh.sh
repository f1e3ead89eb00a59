#!/bin/bash
# End-of-round GPU pass: scripts/gpu_full.sh over every workload (each with its CPU leg), then
# kernel-trace + FETCH_SIZE / WRITE_SIZE profiles of the headline verify, the 4 KiB
# small-chunk batch, the config-3 block-update step and the config-3 UpdateIO batch, each
# summarised into gpurun_out/prof_<tag>/summary.{txt,json} (the json is what bench.py cites).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
WORKLOADS="update updio hostfed shard4m mixed sync" bash scripts/gpu_full.sh || exit 1
prof() {  # tag kernel alg_bytes description workload [bench args]
  local tag=$1 kern=$2 alg=$3 desc=$4 w=$5; shift 5
  bash scripts/profile.sh $w $tag "$@" > gpurun_out/prof_$tag.log 2>&1 || { echo PROF_${tag}_FAIL; exit 1; }
  python3 scripts/summarize_kernels.py gpurun_out/prof_$tag --json $kern $alg "$desc" gpurun_out/prof_$tag/summary.json \
    > /dev/null || exit 1
}
prof headline seg_crc_kernel 8589934592 "bench.py: 8192 x 1 MiB device-resident chunks (BASELINE config 2)" verify --hostfed-extra-gib 0
prof small4k seg_uni_kernel 8589934592 "bench.py --chunks 2097152 --chunk-kib 4: 8 GiB of 4 KiB chunks (uniform small-chunk kernel)" verify --chunks 2097152 --chunk-kib 4 --hostfed-extra-gib 0
prof upd upd_fused_kernel 1228800000 "bench.py --workload update: 100000 x 4 KiB writes into 64 x 64 MiB chunks (fused path)" update
prof updio uio_fast_kernel 1228800000 "bench.py --workload updio: 100000 x 4 KiB UpdateIOs into 64 x 64 MiB chunks (h3c_update_ios_dev, fast branch)" updio
echo REFRESH_OK
