#!/bin/bash
# Round-4 closing pass after the block-update tail change: smoke, every GPU test, the default and update / updio
# bench lines, and the block-update profile (kernel trace + FETCH_SIZE / WRITE_SIZE) summarised for bench.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
WORKLOADS="update updio" bash scripts/gpu_full.sh || exit 1
bash scripts/profile.sh update upd > gpurun_out/prof_upd.log 2>&1 || { echo PROF_upd_FAIL; tail -5 gpurun_out/prof_upd.log; exit 1; }
python3 scripts/summarize_kernels.py gpurun_out/prof_upd --json upd_fused_kernel 1228800000 \
  "bench.py --workload update: 100000 x 4 KiB writes into 64 x 64 MiB chunks (fused path)" gpurun_out/prof_upd/summary.json > /dev/null || exit 1
echo FINAL2_OK
