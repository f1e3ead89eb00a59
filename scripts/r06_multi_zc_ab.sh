#!/bin/bash
# Same-box A/B of h3c_multi_plan_verify in place (the kernels read expected values from and write results into the pinned mirror; shipped) vs copies through a device buffer.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for r in 1 2 3; do
  for v in ship nozc; do
    if [ $v = ship ]; then unset H3C_LIB_PATH; else export H3C_LIB_PATH=$PWD/3fs_amd/_lib/diag/nozc/libh3c_crc.so; fi
    timeout -k 10 120 python -u bench.py --gpus 1 --inproc --devices 0 --steps 200 --warmup 10 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo FAIL $v; tail -20 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['ms_per_step'], d['per_worker'][0]['last_ms'], d['verified'])" | tee -a gpurun_out/r06_multi_zc_ab.txt
  done
done
