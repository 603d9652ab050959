set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_rl
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "bitonic or shuffle or advanced or nips19 or composite or topk or client or fold" > gpurun_out/pytest_gpu${TAG:-x}.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu${TAG:-x}.log; [ $rc -eq 0 ] || exit 1
for rl in 1 0; do FLTEE_BITONIC_REGLEVELS=$rl timeout -k 10 300 python scripts/bench_sort.py --sizes 16,20,24,27 > gpurun_out/sort_${TAG:-x}_rl$rl.jsonl 2>&1 || exit 2; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rl/${TAG:-x} -o run -- python3 scripts/bench_sort.py --sizes 27 --modes 0,2 --reps 2 > gpurun_out/prof_rl_${TAG:-x}.log 2>&1 || exit 3
echo done
