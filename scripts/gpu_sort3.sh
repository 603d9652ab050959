set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "14 1" "13 1" "14 0" "13 0"; do set -- $cfg
  FLTEE_BITONIC_TLOG=$1 FLTEE_BITONIC_STRIDED=$2 timeout -k 10 300 python scripts/bench_sort.py --sizes 20,24,27 > gpurun_out/sort_k_t$1_s$2.jsonl 2>&1 || exit 2
  FLTEE_BITONIC_TLOG=$1 FLTEE_BITONIC_STRIDED=$2 timeout -k 10 300 python scripts/bench_advanced.py --workload c5 --rounds 2 --launches 3 > gpurun_out/adv_k_t$1_s$2.jsonl 2>&1 || exit 3
done
echo done
