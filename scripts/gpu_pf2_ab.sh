set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pf2_ab
mkdir -p $O
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 200 python scripts/bench_sort.py --sizes 24,27 --modes 0,2 --reps 5 > $O/sort_$tag.jsonl 2> $O/$tag.err || return 1
  env "$@" timeout -k 10 200 python bench.py --workload c5 --steps 6 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/c5_$tag.json 2>> $O/$tag.err || return 1
}
run base FLTEE_X=0 || exit 2
run t13 FLTEE_BITONIC_TLOG=13 || exit 3
run t13pf2 FLTEE_BITONIC_TLOG=13 FLTEE_BITONIC_PF2=1 || exit 4
FLTEE_BITONIC_TLOG=13 FLTEE_BITONIC_PF2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "bitonic or shuffle or advanced" > $O/pytest_pf2.log 2>&1 || exit 5
echo done
