#!/bin/bash
# A/B job: the parity tests of the networks on the product library, then
# scripts/ab_env.py over the A/B builds in fl-tee_amd/lib/ab (scripts/ab_build.sh) for
# each workload.  TAG=... WORKLOADS="c5 c4 c3" VARIANTS="name1 name2" bash scripts/gpu_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "${PYTEST_K:-bitonic or advanced or nips19 or shuffle or sort or pad_skip}" > "$OUT/pytest.log" 2>&1 || exit 11
tail -1 "$OUT/pytest.log"
args=""
for v in ${VARIANTS}; do args="$args FLTEE_LIB=fl-tee_amd/lib/ab/libfltee_agg_$v.so"; done
for w in ${WORKLOADS:-c5 c4 c3}; do
  AB_REPS=${AB_REPS:-2} timeout -k 10 900 python -u scripts/ab_env.py $w $args > "$OUT/$w.jsonl" 2> "$OUT/$w.err" || exit 12
  echo "ab $w done"
done
