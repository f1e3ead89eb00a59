#!/bin/bash
# Mixed 64 KiB-64 MiB verify at forced segment sizes (H3C_SEG_BYTES; 0 = the plan's own pick), same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/r06_mixed_seg.txt
: > $out
for sb in 0 131072 262144 524288 1048576; do
  for r in 1 2; do
    if [ $sb = 0 ]; then unset H3C_SEG_BYTES; else export H3C_SEG_BYTES=$sb; fi
    timeout -k 10 200 python -u bench.py --workload mixed --no-cpu-baseline > gpurun_out/r06_mx.json 2>/dev/null || exit 1
    python3 - "$sb" >> $out <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r06_mx.json") if l.startswith("{")][0])
r = d["roofline"]
print(f"seg={sys.argv[1]:8s} value={d['value']} ms={d['ms_per_step']} kernel_us={r.get('kernel_avg_us')} frac={r['frac']} verified={d['verified']}")
PY
  done
done
cat $out
