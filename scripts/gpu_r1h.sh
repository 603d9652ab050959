set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "shuffle or nips19 or network or fused or bitonic or repeatable" > $O/pytest.log 2>&1 || exit 2
timeout -k 10 300 python scripts/bench_sort.py --sizes 20,24,27 --modes 0,2 --reps 5 > $O/sort.jsonl 2> $O/sort.err || exit 3
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/c4.json 2> $O/c4.err || exit 4
echo done
