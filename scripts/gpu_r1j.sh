set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "safe_aggregate or nips19" > $O/pytest.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --workload c4 --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/prof_c4.log 2>&1 || exit 3
echo done
