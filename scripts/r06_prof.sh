#!/bin/bash
# Round-6 profile pass: kernel trace + FETCH_SIZE / WRITE_SIZE passes per workload, each summarised for
# bench.py (profiles/r06_<tag>_pmc_summary.json via scripts/summarize_kernels.py --json).
# usage: TAGS="updio mixed" scripts/r06_prof.sh   (default: all)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
prof() {  # tag kernel alg_bytes description workload [bench args]
  local tag=$1 kern=$2 alg=$3 desc=$4 w=$5; shift 5
  case " ${TAGS:-headline shard4m mixed updio} " in *" $tag "*) ;; *) return 0 ;; esac
  bash scripts/profile.sh $w r06_$tag "$@" > gpurun_out/prof_r06_$tag.log 2>&1 || { echo PROF_${tag}_FAIL; tail -5 gpurun_out/prof_r06_$tag.log; exit 1; }
  python3 scripts/summarize_kernels.py gpurun_out/prof_r06_$tag --json $kern $alg "$desc" gpurun_out/prof_r06_$tag/summary.json \
    > /dev/null || exit 1
  echo "$tag ok"
}
NOX="--hostfed-extra-gib 0 --update-extra 0 --shard4m-extra 0 --inproc-extra 0"
prof headline seg_crc_kernel 8589934592 "bench.py: 8192 x 1 MiB device-resident chunks (BASELINE config 2), no sub-passes" verify $NOX
prof shard4m seg_crc_kernel 34359738368 "bench.py --chunks 8192 --chunk-kib 4096: 8192 x 4 MiB = 32 GiB (BASELINE config 4's per-GPU share at 8 GPUs; the default line's shard4m object)" verify --chunks 8192 --chunk-kib 4096 $NOX
prof mixed seg_crc_kernel 8620183509 "bench.py --workload mixed: 8 GiB of 64 KiB-64 MiB chunks, 10% ragged, packed unaligned" mixed
KT_STEPS=60 KT_WARMUP=20 prof updio uio_afused_kernel 1228800000 "bench.py --workload updio --updio-headline-only: 100000 x 4 KiB UpdateIOs into 64 x 64 MiB chunks, 4 rotating op tables (aligned sub-branch), the timed leg only" updio --updio-headline-only
echo R06PROF_OK
