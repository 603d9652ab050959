set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r1b/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/r1b/pytest_gpu.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 600 python bench.py --extra c1,c3 --no-e2e > gpurun_out/r1b/bench.json 2> gpurun_out/r1b/bench.err || exit 3
echo done
