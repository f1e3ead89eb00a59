#!/bin/bash
# End-of-round GPU pass: scripts/gpu_full.sh over every workload with the headline profile,
# then kernel-trace + FETCH_SIZE / WRITE_SIZE profiles of the 4 KiB small-chunk batch and of
# the config-3 update step, each summarised into gpurun_out/prof_<tag>/summary*.{txt,json}.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
WORKLOADS="update updio hostfed shard4m mixed" PROFILE=1 bash scripts/gpu_full.sh || exit 1
bash scripts/profile.sh verify small4k --chunks 2097152 --chunk-kib 4 --hostfed-extra-gib 0 > gpurun_out/prof_small4k.log 2>&1 || { echo PROF_SMALL_FAIL; exit 1; }
python3 scripts/summarize_kernels.py gpurun_out/prof_small4k --json seg_quad_kernel 8589934592 \
  "bench.py --chunks 2097152 --chunk-kib 4: 8 GiB of 4 KiB chunks (4-lane small-chunk kernel)" \
  gpurun_out/prof_small4k/summary.json > /dev/null || exit 1
bash scripts/profile.sh update upd > gpurun_out/prof_upd.log 2>&1 || { echo PROF_UPD_FAIL; exit 1; }
python3 scripts/summarize_kernels.py gpurun_out/prof_upd --json upd_delta_kernel 1228800000 \
  "bench.py --workload update: 100000 x 4 KiB writes into 64 x 64 MiB chunks" \
  gpurun_out/prof_upd/summary.json > /dev/null || exit 1
echo REFRESH_OK
