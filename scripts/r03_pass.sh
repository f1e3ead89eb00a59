#!/bin/bash
# Round-3 GPU pass: GPU tests, then A/B of this round's kernel changes against variant libraries
# (3fs_amd/_lib/variants/lib_<v>.so), the benches, and the probes.  Every step has its own time
# limit and the first failure ends the pass.  STEPS selects steps (default: all).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
T=${TAG:-r03}
want() { [ -z "$STEPS" ] || [[ " $STEPS " == *" $1 "* ]]; }
jq1() { python -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d.get('ms_per_step'), d['roofline']['achieved'], d['roofline']['kernel_avg_us'], d['verified'])"; }
if want tests; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { echo TESTS_FAIL; exit 1; }
fi
if want updio_ab; then
  for rep in 1 2; do
    for v in cur ${UPDIO_VARIANTS:-prefold}; do
      lib=$R/3fs_amd/_lib/libh3c_crc.so; [ "$v" != cur ] && lib=$R/3fs_amd/_lib/variants/lib_$v.so
      echo -n "$v rep=$rep " >> gpurun_out/${T}_updio_ab.txt
      H3C_LIB_PATH=$lib timeout -k 5 120 python bench.py --workload updio --no-cpu-baseline 2>/dev/null | jq1 >> gpurun_out/${T}_updio_ab.txt || { echo UPDIO_AB_FAIL; exit 1; }
    done
  done
fi
if want small_ab; then
  for rep in 1 2; do
    for kib in 4 8; do
      for v in cur ${SMALL_VARIANTS:-uni4}; do
        lib=$R/3fs_amd/_lib/libh3c_crc.so; [ "$v" != cur ] && lib=$R/3fs_amd/_lib/variants/lib_$v.so
        echo -n "$v ${kib}KiB rep=$rep " >> gpurun_out/${T}_small_ab.txt
        H3C_LIB_PATH=$lib timeout -k 5 120 python bench.py --chunks $((8388608 / kib)) --chunk-kib $kib --no-cpu-baseline --hostfed-extra-gib 0 --steps 20 --warmup 3 2>/dev/null | jq1 >> gpurun_out/${T}_small_ab.txt || { echo SMALL_AB_FAIL; exit 1; }
      done
    done
  done
fi
if want bench; then
  timeout -k 10 200 python bench.py > gpurun_out/${T}_bench.jsonl 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; exit 1; }
fi
if want bench_n2; then
  timeout -k 10 240 python bench.py --gpus 2 --steps 10 --warmup 2 --cpu-seconds 2 > gpurun_out/${T}_bench_n2.jsonl 2> gpurun_out/${T}_bench_n2.err || { echo BENCH_N2_FAIL; exit 1; }
fi
if want update; then
  timeout -k 10 120 python bench.py --workload update > gpurun_out/${T}_bench_update.jsonl 2>&1 || { echo UPDATE_FAIL; exit 1; }
fi
if want updio; then
  timeout -k 10 120 python bench.py --workload updio > gpurun_out/${T}_bench_updio.jsonl 2>&1 || { echo UPDIO_FAIL; exit 1; }
fi
if want rmwphase; then
  timeout -k 10 150 ./scripts/rmwphase > gpurun_out/${T}_rmwphase.txt 2>&1 || { echo RMWPHASE_FAIL; exit 1; }
fi
echo PASS_OK
