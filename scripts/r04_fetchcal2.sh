#!/bin/bash
# r04 #4 follow-up: which load shape / policy removes the 4-lane rows' line re-fetch (the probe only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04cal2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
REQ="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
timeout -s KILL 60 $R/scripts/fetchcal > $O/plain_run.log 2>&1 || { echo RUN_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $REQ -d $O/cal_req -o p --output-format csv -- $R/scripts/fetchcal > $O/cal_req.log 2>&1 || { echo CAL_REQ_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/cal_hit -o p --output-format csv -- $R/scripts/fetchcal > $O/cal_hit.log 2>&1 || { echo CAL_HIT_FAIL; exit 1; }
echo CAL2_OK
