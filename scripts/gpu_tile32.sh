set -o pipefail
cd $GRAFT_REPO_ROOT
FLTEE_BITONIC_TILE32=1 timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "bitonic or shuffle or advanced or nips19" > gpurun_out/pytest_gpu${TAG:-x}.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu${TAG:-x}.log; [ $rc -eq 0 ] || exit 1
for t in 1 0; do FLTEE_BITONIC_TILE32=$t timeout -k 10 300 python scripts/bench_sort.py --sizes 22,24,27 > gpurun_out/sort_${TAG:-x}_t32$t.jsonl 2>&1 || exit 2
FLTEE_BITONIC_TILE32=$t timeout -k 10 300 python scripts/bench_advanced.py --workload c5 --rounds 2 --launches 3 > gpurun_out/adv_${TAG:-x}_t32$t.jsonl 2>&1 || exit 3; done
export TMPDIR=/tmp
FLTEE_BITONIC_TILE32=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_t32_${TAG:-x} -o run -- python3 scripts/bench_sort.py --sizes 27 --modes 0 --reps 2 > gpurun_out/prof_t32_${TAG:-x}.log 2>&1 || exit 4
echo done
