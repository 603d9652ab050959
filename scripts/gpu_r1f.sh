set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1f
mkdir -p $O
for c in 0 4 5; do
  for dd in 0 2 4; do
    FLTEE_FOLD_CLOG=$c FLTEE_FOLD_DEPTH=$dd timeout -k 10 120 python scripts/fold_ab.py c3 >> $O/fold_c3.jsonl 2>> $O/fold.err || exit 3
  done
done
for t in 0 1 0 1; do
  FLTEE_BITONIC_TILE32=$t timeout -k 10 200 python scripts/bench_sort.py --sizes 20,24,27 --modes 0,2 --reps 5 >> $O/sort_tile32_$t.jsonl 2>> $O/sort.err || exit 4
done
FLTEE_BITONIC_TILE32=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "bitonic or shuffle or fused or advanced or nips19" > $O/pytest_tile32.log 2>&1 || exit 5
echo done
