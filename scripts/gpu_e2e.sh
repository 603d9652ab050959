set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "ecall or server or wire or client" > gpurun_out/pytest_gpu${TAG:-x}.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu${TAG:-x}.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --steps 10 --no-extra --no-cpu-baseline > gpurun_out/bench_e2e_${TAG:-x}.json 2> gpurun_out/bench_e2e_${TAG:-x}.err || exit 2
echo done
