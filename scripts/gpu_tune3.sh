set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu5.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu5.log
timeout -k 10 300 python scripts/bench_sort.py --sizes 16,20,24,27 > gpurun_out/sort_g.jsonl 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4b -o run -- python3 bench.py --workload c4 --steps 5 --warmup 1 --no-extra --no-cpu-baseline --no-e2e > gpurun_out/prof_c4b.log 2>&1 || exit 2
echo done
