#!/bin/bash
# One gpurun job that regenerates the round's GPU evidence (run under gpurun from the
# repo root):  TAG=r03 [TESTS=1] [BENCH=1] [PROFILE="ns c1 c3 c4 mnist100"] [PMC="ns"] \
#              [SQ="c4 c5"] [AB="c4" ABV="FLTEE_LIB=..."] bash scripts/gpu_evidence.sh
# Every GPU step has its own time limit and the steps stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
TAG=${TAG:-rxx}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_X--x} -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1 || exit 11
  tail -3 "$OUT/pytest_gpu.log"
fi
# A/B of library builds in one process per variant: AB="c4 c5" ABV="FLTEE_LIB=fl-tee_amd/lib/ab/x.so"
for w in ${AB}; do
  timeout -k 10 600 python -u scripts/ab_env.py "$w" ${ABV} > "$OUT/ab_$w.jsonl" 2> "$OUT/ab_$w.err" || exit 22
  echo "ab $w"
done
# A/B of a runtime hook in one process: ABH="mnist100:fltee_debug_set_dense_variant:0 44 45"
for spec in ${ABH:+"$ABH"}; do
  IFS=: read -r w hook vals <<< "$spec"
  timeout -k 10 600 python -u scripts/ab_hook.py "$w" "$hook" $vals > "$OUT/abh_${w}_${hook}.jsonl" 2> "$OUT/abh_$w.err" || exit 23
  echo "abh $w $hook"
done
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} --detail "$OUT/bench_detail.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 12
  tail -c 600 "$OUT/bench.json"; echo
fi
for w in ${PROFILE}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o run \
      -- python3 bench.py --workload "$w" --steps 20 --warmup 3 --no-extra --no-cpu-baseline \
      --no-e2e --detail "$OUT/prof_$w.detail.json" > "$OUT/prof_$w.log" 2>&1 || exit 13
  echo "profiled $w"
done
for w in ${PMC}; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$w" -o run \
      -- python3 bench.py --workload "$w" --steps 10 --warmup 2 --no-extra --no-cpu-baseline \
      --no-e2e --detail "" > "$OUT/pmc_fetch_$w.log" 2>&1 || exit 14
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$w" -o run \
      -- python3 bench.py --workload "$w" --steps 10 --warmup 2 --no-extra --no-cpu-baseline \
      --no-e2e --detail "" > "$OUT/pmc_write_$w.log" 2>&1 || exit 15
  echo "pmc $w"
done
# SQ counters per kernel (one pass of <= 8 SQ counters each, its own run)
SQ1=${SQ1:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT}
SQ2=${SQ2:-SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR}
SQ3=${SQ3:-SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES}
SQC=${SQC:-SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ}
for w in ${SQ}; do
  timeout -s KILL 150 rocprofv3 --pmc ${SQ1} --output-format csv -d "$OUT/sq1_$w" -o run \
      -- python3 bench.py --workload "$w" --steps 6 --warmup 1 --no-extra --no-cpu-baseline \
      --no-e2e --detail "" > "$OUT/sq1_$w.log" 2>&1 || exit 18
  timeout -s KILL 150 rocprofv3 --pmc ${SQ2} --output-format csv -d "$OUT/sq2_$w" -o run \
      -- python3 bench.py --workload "$w" --steps 6 --warmup 1 --no-extra --no-cpu-baseline \
      --no-e2e --detail "" > "$OUT/sq2_$w.log" 2>&1 || exit 19
  timeout -s KILL 150 rocprofv3 --pmc ${SQ3} --output-format csv -d "$OUT/sq3_$w" -o run \
      -- python3 bench.py --workload "$w" --steps 6 --warmup 1 --no-extra --no-cpu-baseline \
      --no-e2e --detail "" > "$OUT/sq3_$w.log" 2>&1 || exit 20
  timeout -s KILL 150 rocprofv3 --pmc ${SQC} --output-format csv -d "$OUT/sqc_$w" -o run \
      -- python3 bench.py --workload "$w" --steps 6 --warmup 1 --no-extra --no-cpu-baseline \
      --no-e2e --detail "" > "$OUT/sqc_$w.log" 2>&1 || exit 21
  echo "sq $w"
done
if [ "${ORAM:-0}" = 1 ]; then  # the tree Path ORAM (scripts/oram_probe.py): timing + SQ passes
  timeout -k 10 120 python3 -u scripts/oram_probe.py 10 5089 50890 > "$OUT/oram_probe.log" 2>&1 || exit 24
  cat "$OUT/oram_probe.log"
  for p in 1 2 3; do
    eval "cs=\$SQ$p"
    timeout -s KILL 120 rocprofv3 --pmc ${cs} --output-format csv -d "$OUT/sq${p}_oram" -o run \
        -- python3 scripts/oram_probe.py 3 5089 50890 > "$OUT/sq${p}_oram.log" 2>&1 || exit 25
  done
  echo "oram"
fi
if [ "${AESPROF:-0}" = 1 ]; then  # the constant-time AES-CTR kernel (scripts/bench_aes.py shapes)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_aes" -o run \
      -- python3 scripts/bench_aes.py > "$OUT/prof_aes.log" 2>&1 || exit 17
  echo "profiled aes"
fi
if [ "${CABI:-0}" = 1 ]; then  # the C-ABI multi-GPU eid over the visible GPUs (1-rank RCCL on one)
  timeout -k 10 300 python -u scripts/ecall_multi_bench.py > "$OUT/c_abi_multi_gpu.json" 2> "$OUT/c_abi_multi_gpu.err" || exit 16
  echo "c_abi"
fi
echo done
