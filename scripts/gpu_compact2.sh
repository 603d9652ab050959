set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_c5${TAG:-x}
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "advanced or optimized or ecall or wire or client" > gpurun_out/pytest_gpu${TAG:-x}.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu${TAG:-x}.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/bench_advanced.py --workload c5 --rounds 2 --launches 3 > gpurun_out/adv_${TAG:-x}.jsonl 2>&1 || exit 2
timeout -k 10 300 python scripts/bench_advanced.py --workload c3 --rounds 5 --launches 20 > gpurun_out/adv_c3_${TAG:-x}.jsonl 2>&1 || exit 3
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5${TAG:-x} -o run -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-extra --no-cpu-baseline --no-e2e > gpurun_out/prof_c5${TAG:-x}.log 2>&1 || exit 4
echo done
