set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tiles_ab
mkdir -p $O
for mt in 8 7 6 5; do
FLTEE_BITONIC_MINTILES_LOG=$mt timeout -k 10 120 python scripts/bench_sort.py --sizes 16,18,20,21,22,23 --modes 0 --reps 7 > $O/mt$mt.jsonl 2> $O/mt$mt.err || exit 2
FLTEE_BITONIC_MINTILES_LOG=$mt timeout -k 10 200 python bench.py --workload c3 --steps 20 --no-extra --no-cpu-baseline --no-e2e > $O/c3_mt$mt.json 2>> $O/mt$mt.err || exit 3
done
timeout -k 10 120 python bench.py --workload c1 --steps 20 --no-extra --no-cpu-baseline --no-e2e > $O/c1.json 2> $O/c1.err || exit 4
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "sparse or scatter or non_oblivious" > $O/pytest.log 2>&1 || exit 5
echo done
