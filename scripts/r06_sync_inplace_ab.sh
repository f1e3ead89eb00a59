#!/bin/bash
# Synchronous batch API (batch_sync): results written in place into the pinned lease (shipped) vs copied back
# from the device arena.  The whole GPU suite on the working tree, then the sync workload per library, same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06_sip_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/r06_sip_tests.log; exit 1; }
tail -1 gpurun_out/r06_sip_tests.log
out=gpurun_out/r06_sync_inplace_ab.txt
: > $out
for rep in 1 2; do
  for v in ship noinplace; do
    lib=$PWD/3fs_amd/_lib/libh3c_crc.so; [ $v = noinplace ] && lib=$PWD/3fs_amd/_lib/diag/noinplace/libh3c_crc.so
    H3C_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --workload sync --no-cpu-baseline > gpurun_out/r06_sip.json 2>gpurun_out/r06_sip.err || { echo BENCH_FAIL; tail gpurun_out/r06_sip.err; exit 1; }
    python3 - "$v" >> $out <<'PY'
import json, sys
d = [json.loads(l) for l in open("gpurun_out/r06_sip.json") if l.startswith("{")][0]
rows = d.get("rows") or d.get("sizes") or []
print(sys.argv[1], json.dumps(rows)[:900])
PY
  done
done
cat $out
