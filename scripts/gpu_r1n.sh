set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "dense or headline or clip or decrypt or parallel" > $O/pytest.log 2>&1 || exit 2
for w in mnist30 mnist100; do
  timeout -k 10 300 python bench.py --workload $w --steps 200 --warmup 10 --no-extra --no-cpu-baseline --no-e2e > $O/bench_$w.json 2> $O/bench_$w.err || exit 4
done
echo done
