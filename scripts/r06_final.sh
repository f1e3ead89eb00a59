#!/bin/bash
# Round-6 closing pass: the whole GPU test suite, smoke(), then the default bench line (driver form).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06z_gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/r06z_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06z_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r06z_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r06z_smoke.log; exit 1; }
tail -1 gpurun_out/r06z_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r06z_bench_default.json 2> gpurun_out/r06z_bench_default.err || { echo BENCH_FAIL; tail -20 gpurun_out/r06z_bench_default.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06z_bench_default.json") if l.startswith("{")][0])
print("headline", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["verified"])
for k in ("update", "shard4m", "inproc", "hostfed"):
    o = d.get(k) or {}
    print(k, o.get("value"), o.get("ms_per_step"), o.get("verified"), (o.get("roofline") or {}).get("frac"), (o.get("roofline") or {}).get("kernel_avg_us"))
PY
