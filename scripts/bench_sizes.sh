#!/bin/bash
# Verify throughput across chunk sizes / alignment (kernel GB/s and frac per line).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-sizes}
timeout -k 10 200 python bench.py --workload mixed > gpurun_out/${TAG}_mixed.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --chunks 131072 --chunk-kib 64 --no-cpu-baseline > gpurun_out/${TAG}_64k.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_1m.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --chunks 2048 --chunk-kib 4096 --no-cpu-baseline > gpurun_out/${TAG}_4m.log 2>&1 || exit 1
for f in mixed 64k 1m 4m; do
  tail -1 gpurun_out/${TAG}_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['verified'])"
done
