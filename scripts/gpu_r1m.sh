set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1m
mkdir -p $O
export TMPDIR=/tmp
for w in mnist30 mnist100; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 50 --warmup 5 --no-extra --no-cpu-baseline --no-e2e > $O/prof_$w.log 2>&1 || exit 3
  timeout -k 10 300 python bench.py --workload $w --steps 200 --warmup 10 --no-extra --no-cpu-baseline --no-e2e > $O/bench_$w.json 2> $O/bench_$w.err || exit 4
done
echo done
