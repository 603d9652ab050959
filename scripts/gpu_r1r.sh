set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "bitonic or shuffle or fused or advanced or nips19 or repeatable" > $O/pytest.log 2>&1 || exit 2
for t in 1 0 1 0; do
  FLTEE_BITONIC_DIRECT_SORT8=$t timeout -k 10 300 python bench.py --workload c3 --steps 100 --warmup 10 --no-extra --no-cpu-baseline --no-e2e > $O/c3_$t.json 2>> $O/c3.err || exit 3
  FLTEE_BITONIC_DIRECT_SORT8=$t timeout -k 10 300 python scripts/bench_sort.py --sizes 20 --modes 0,2 --reps 10 >> $O/sort20_$t.jsonl 2>> $O/sort.err || exit 4
  cat $O/c3_$t.json >> $O/c3_$t.all
done
echo done
