set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/strided
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "bitonic or shuffle or advanced or network or sharded or nips19 or repeatable" > $O/pytest.log 2>&1 || exit 2
for x in a b; do timeout -k 10 200 python scripts/debug_direct.py $O/on_$x.json 2> $O/m.err || exit 3; done
FLTEE_BITONIC_DIRECT_STRIDED=0 timeout -k 10 200 python scripts/debug_direct.py $O/off.json 2>> $O/m.err || exit 3
timeout -k 10 200 python scripts/bench_sort.py --sizes 24,27 --modes 0,2 --reps 5 > $O/sort_on.jsonl 2>> $O/m.err || exit 4
FLTEE_BITONIC_DIRECT_STRIDED=0 timeout -k 10 200 python scripts/bench_sort.py --sizes 24,27 --modes 0,2 --reps 5 > $O/sort_off.jsonl 2>> $O/m.err || exit 4
for w in c4 c5; do timeout -k 10 200 python bench.py --workload $w --steps 6 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/$w.json 2>> $O/m.err || exit 5; done
echo done
