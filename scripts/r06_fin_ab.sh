#!/bin/bash
# one finalize launch with its loads issued before the table build, against HEAD's two launches:
# the whole GPU test suite on the working tree, then mixed / 4 MiB / 1 MiB verify, same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06_fin_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/r06_fin_tests.log; exit 1; }
tail -1 gpurun_out/r06_fin_tests.log
out=gpurun_out/r06_fin_ab.txt
: > $out
for rep in 1 2; do
  for v in new base; do
    lib=$PWD/3fs_amd/_lib/libh3c_crc.so; [ $v = base ] && lib=$PWD/3fs_amd/_lib/diag/base/libh3c_crc.so
    for w in "mixed" "verify --chunks 8192 --chunk-kib 4096" "verify"; do
      H3C_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --hostfed-extra-gib 0 --update-extra 0 --shard4m-extra 0 --inproc-extra 0 > gpurun_out/r06_fin.json 2>/dev/null || exit 1
      python - "$v $w" >> $out <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r06_fin.json") if l.startswith("{")][0])
r = d["roofline"]
print(f"{sys.argv[1]:48s} value={d['value']} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r.get('kernel_avg_us')} frac={r['frac']}")
PY
    done
  done
done
cat $out
