set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu2.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu2.log
for r in 4 5 6; do
  FLTEE_BITONIC_MAXR=$r timeout -k 10 300 python scripts/bench_sort.py --sizes 20,24,27 > gpurun_out/sort_r$r.jsonl 2>&1 || exit 1
done
timeout -k 10 400 python bench.py > gpurun_out/bench_r01b.json 2> gpurun_out/bench_r01b.err || exit 2
echo done
