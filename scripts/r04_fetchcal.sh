#!/bin/bash
# calibrate FETCH_SIZE for the 4-lane x 64-byte row shape.  Memory-side read
# requests by size (TCC_EA0_RDREQ_{32B,64B,128B}_sum, TCC_EA0_RDREQ_sum) and FETCH_SIZE, each in
# its own --pmc pass, for (1) scripts/fetchcal (three shapes, 8 GiB each, known byte count) and
# (2) the engine's 4 KiB uniform verify and 1 MiB headline verify.  Outputs: gpurun_out/r04cal/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04cal
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
REQ="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/cal_fetch -o p --output-format csv -- $R/scripts/fetchcal > $O/cal_fetch.log 2>&1 || { echo CAL_FETCH_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $REQ -d $O/cal_req -o p --output-format csv -- $R/scripts/fetchcal > $O/cal_req.log 2>&1 || { echo CAL_REQ_FAIL; exit 1; }
B="python3 $R/bench.py --hostfed-extra-gib 0 --no-cpu-baseline --steps 3 --warmup 1"
timeout -s KILL 150 rocprofv3 --pmc $REQ -d $O/small_req -o p --output-format csv -- $B --chunks 2097152 --chunk-kib 4 > $O/small_req.log 2>&1 || { echo SMALL_REQ_FAIL; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/small_fetch -o p --output-format csv -- $B --chunks 2097152 --chunk-kib 4 > $O/small_fetch.log 2>&1 || { echo SMALL_FETCH_FAIL; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $REQ -d $O/head_req -o p --output-format csv -- $B > $O/head_req.log 2>&1 || { echo HEAD_REQ_FAIL; exit 1; }
echo CAL_OK
