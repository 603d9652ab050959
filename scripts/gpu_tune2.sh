set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu4.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu4.log
timeout -k 10 300 python scripts/bench_dense.py > gpurun_out/dense_variants.jsonl 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_sort.py --sizes 20,24,27 > gpurun_out/sort_f.jsonl 2>&1 || exit 2
echo done
