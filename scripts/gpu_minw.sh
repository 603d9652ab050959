set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/minw
mkdir -p $O
for w in 4 3 2 1; do
FLTEE_BITONIC_MINW_LOG=$w timeout -k 10 200 python scripts/bench_sort.py --sizes 24,27 --modes 0,2 --reps 5 > $O/sort_w$w.jsonl 2> $O/w$w.err || exit 2
done
FLTEE_BITONIC_MINW_LOG=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "bitonic or shuffle or compaction_c5" > $O/pytest.log 2>&1 || exit 3
echo done
