set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1l
mkdir -p $O
for t in 0 1 0 1; do
  FLTEE_BITONIC_SORT32=$t timeout -k 10 200 python scripts/bench_sort.py --sizes 24,27 --modes 0,2 --reps 5 >> $O/sort32_$t.jsonl 2>> $O/sort.err || exit 2
done
FLTEE_BITONIC_SORT32=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "bitonic or shuffle or fused or advanced or nips19" > $O/pytest_sort32.log 2>&1 || exit 3
FLTEE_BITONIC_SORT32=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-e2e > $O/prof_c5.log 2>&1 || exit 4
echo done
