set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu3.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu3.log
timeout -k 10 300 python scripts/bench_sort.py --sizes 16,18,20,24,27 > gpurun_out/sort_e.jsonl 2>&1 || exit 1
export TMPDIR=/tmp
for w in c1 c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$w -o run -- python3 bench.py --workload $w --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-e2e > gpurun_out/prof_$w.log 2>&1 || exit 2
done
timeout -k 10 500 python bench.py > gpurun_out/bench_r01c.json 2> gpurun_out/bench_r01c.err || exit 3
echo done
