#!/bin/bash
# The segment-size pick with a per-segment cost against the balance-only pick: the whole GPU test suite on the
# working tree, then mixed / 1 MiB / 4 MiB / 4 KiB verify, same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06_segpick_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/r06_segpick_tests.log; exit 1; }
tail -1 gpurun_out/r06_segpick_tests.log
out=gpurun_out/r06_segpick_ab.txt
: > $out
for rep in 1 2; do
  for v in new base; do
    lib=$PWD/3fs_amd/_lib/libh3c_crc.so; [ $v = base ] && lib=$PWD/3fs_amd/_lib/diag/base/libh3c_crc.so
    for w in "mixed" "verify" "verify --chunks 8192 --chunk-kib 4096" "verify --chunks 2097152 --chunk-kib 4"; do
      H3C_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --hostfed-extra-gib 0 --update-extra 0 --shard4m-extra 0 --inproc-extra 0 > gpurun_out/r06_sp.json 2>/dev/null || exit 1
      python - "$v $w" >> $out <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r06_sp.json") if l.startswith("{")][0])
r = d["roofline"]
print(f"{sys.argv[1]:52s} value={d['value']} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r.get('kernel_avg_us')} frac={r['frac']}")
PY
    done
  done
done
cat $out
