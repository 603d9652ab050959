# gpurun job: selected GPU tests (PYTEST_K / FILES) then short bench lines per workload (WL)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
if [ -n "$FILES" ]; then
  timeout -k 10 600 python -u -m pytest $FILES ${PYTEST_K:+-k "$PYTEST_K"} -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 11; }
  tail -2 $OUT/pytest.log
fi
for w in $WL; do
  timeout -k 10 300 python -u bench.py --workload $w --steps ${STEPS:-50} --warmup 5 --no-extra --no-cpu-baseline --no-e2e > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 12; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1]); print('$w', d['ms_per_step'], d['value'])"
done
