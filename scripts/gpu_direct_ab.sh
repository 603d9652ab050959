set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/direct_ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_client.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 2
for tag in on off; do
  if [ $tag = off ]; then export FLTEE_BITONIC_DIRECT=0; fi
  timeout -k 10 200 python scripts/bench_sort.py --sizes 20,22,24,27 --modes 0,2 --reps 5 > $O/sort_$tag.jsonl 2> $O/$tag.err || exit 3
  for w in c3 c4 c5; do
    timeout -k 10 200 python bench.py --workload $w --steps 6 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/${w}_$tag.json 2>> $O/$tag.err || exit 4
  done
done
echo done
