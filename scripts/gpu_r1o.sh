set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1o
mkdir -p $O
timeout -k 10 300 python scripts/bench_dense.py --n 30 --d 50890 --rounds 7 --launches 50 > $O/dense_n30.jsonl 2> $O/d30.err || exit 2
timeout -k 10 300 python scripts/bench_dense.py --n 100 --d 50890 --rounds 7 --launches 50 > $O/dense_n100.jsonl 2> $O/d100.err || exit 3
timeout -k 10 300 python scripts/bench_dense.py --n 300 --d 44964 --rounds 5 --launches 20 > $O/dense_n300.jsonl 2> $O/d300.err || exit 4
echo done
