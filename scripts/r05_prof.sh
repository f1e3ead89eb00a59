#!/bin/bash
# Round-5 profile pass: kernel trace + FETCH_SIZE / WRITE_SIZE passes, each summarised for bench.py
# (profiles/r05_<tag>_pmc_summary.json via scripts/summarize_kernels.py --json).
# usage: TAGS="updio upd" scripts/r05_prof.sh   (default: all)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
prof() {  # tag kernel alg_bytes description workload [bench args]
  local tag=$1 kern=$2 alg=$3 desc=$4 w=$5; shift 5
  case " ${TAGS:-headline small4k upd updio shard4m} " in *" $tag "*) ;; *) return 0 ;; esac
  bash scripts/profile.sh $w $tag "$@" > gpurun_out/prof_$tag.log 2>&1 || { echo PROF_${tag}_FAIL; tail -5 gpurun_out/prof_$tag.log; exit 1; }
  python3 scripts/summarize_kernels.py gpurun_out/prof_$tag --json $kern $alg "$desc" gpurun_out/prof_$tag/summary.json \
    > /dev/null || exit 1
  echo "$tag ok"
}
prof headline seg_crc_kernel 8589934592 "bench.py: 8192 x 1 MiB device-resident chunks (BASELINE config 2), no sub-passes" verify --hostfed-extra-gib 0 --update-extra 0
prof small4k seg_uni_kernel 8589934592 "bench.py --chunks 2097152 --chunk-kib 4: 8 GiB of 4 KiB chunks (uniform small-chunk kernel, plain sub-line loads)" verify --chunks 2097152 --chunk-kib 4 --hostfed-extra-gib 0
KT_STEPS=60 KT_WARMUP=20 prof upd upd_fused_kernel 1228800000 "bench.py --workload update: 100000 x 4 KiB writes into 64 x 64 MiB chunks (fused path)" update
KT_STEPS=60 KT_WARMUP=20 prof updio uio_afused_kernel 1228800000 "bench.py --workload updio: 100000 x 4 KiB UpdateIOs into 64 x 64 MiB chunks (h3c_update_ios_dev, aligned sub-branch)" updio
prof shard4m seg_crc_kernel 68719476736 "bench.py --workload shard4m: passes of 16384 x 4 MiB chunks (BASELINE config 4)" shard4m
echo R05PROF_OK
