set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1k
mkdir -p $O
timeout -k 10 300 python scripts/bench_advanced.py --workload c5 --rounds 3 --launches 3 > $O/adv_c5.jsonl 2> $O/adv_c5.err || exit 2
timeout -k 10 300 python scripts/bench_advanced.py --workload c3 --rounds 5 --launches 20 > $O/adv_c3.jsonl 2> $O/adv_c3.err || exit 3
echo done
