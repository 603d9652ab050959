set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ns -o run -- python3 bench.py --steps 30 --no-extra --no-cpu-baseline --no-e2e > $O/prof_ns.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/pmc_fetch.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/pmc_write.log 2>&1 || exit 6
for w in c1 c3 c4 c5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/prof_$w.log 2>&1 || exit 7
done
echo done
