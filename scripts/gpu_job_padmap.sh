#!/bin/bash
# Round-3 job: the networks' parity tests, then the pad-skip levels A/B in one process
# (2: pad-only units inside the mixed block, 1: stage blocks only) at C5 and C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
OUT=gpurun_out/${TAG:-padmap}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5_full.py -x -q --timeout 300 \
    --timeout-method thread -k "${PYTEST_K:-bitonic or advanced or sort or pad_skip or fused or c5}" \
    > "$OUT/pytest.log" 2>&1 || exit 11
tail -1 "$OUT/pytest.log"
for w in ${WORKLOADS:-c5 c3}; do
  AB_REPS=${AB_REPS:-3} timeout -k 10 400 python -u scripts/ab_hook.py $w fltee_debug_set_pad_skip 2 1 \
      > "$OUT/ab_$w.jsonl" 2> "$OUT/ab_$w.err" || exit 12
  echo "ab $w done"
done
