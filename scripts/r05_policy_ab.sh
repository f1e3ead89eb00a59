#!/bin/bash
# Round-5 write-back / load policy A/B on every config-3 kernel (profiles/r05s_rmw_policy_ab.txt):
# the shipped library against build variants (scripts/build_variant.sh), each branch forced by its hook.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
V=${VARIANTS:-psall}
VARIANTS="$V" WORKLOAD=updio REPS=2 ARGS="--steps 100 --warmup 30" bash scripts/ab_variants.sh > gpurun_out/r05u_ab_updio.txt 2>&1 || exit 1
VARIANTS="$V" WORKLOAD=update REPS=2 ARGS="--steps 100 --warmup 30" bash scripts/ab_variants.sh > gpurun_out/r05u_ab_update.txt 2>&1 || exit 1
H3C_UPD_ALIGNED=1 VARIANTS="$V" WORKLOAD=updio REPS=2 ARGS="--steps 60 --warmup 20" bash scripts/ab_variants.sh > gpurun_out/r05u_ab_fastchain.txt 2>&1 || exit 1
H3C_UPD_FAST=1 VARIANTS="$V" WORKLOAD=updio REPS=2 ARGS="--steps 40 --warmup 10" bash scripts/ab_variants.sh > gpurun_out/r05u_ab_general.txt 2>&1 || exit 1
echo DONE
