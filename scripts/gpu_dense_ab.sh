set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dense_ab
timeout -k 10 300 python scripts/bench_dense.py --rounds 7 --launches 20 > gpurun_out/dense_ab/ab.jsonl 2> gpurun_out/dense_ab/ab.err || exit 2
timeout -k 10 300 python bench.py --no-extra --no-e2e > gpurun_out/dense_ab/bench.json 2> gpurun_out/dense_ab/bench.err || exit 3
echo done
