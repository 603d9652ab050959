set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r01
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -k "k0_quirk or advanced" > gpurun_out/pytest_k0.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_k0.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01/trace -o run -- python3 bench.py --steps 20 --no-extra --no-cpu-baseline > gpurun_out/prof_r01/trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_r01/fetch -o run -- python3 bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline > gpurun_out/prof_r01/fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_r01/write -o run -- python3 bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline > gpurun_out/prof_r01/write.log 2>&1 || exit 4
echo done
