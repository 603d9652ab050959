# gpurun job: selected GPU parity tests (PYTEST_K over FILES), then one-process hook A/Bs
# (HOOKAB="c5:fltee_debug_set_fold_compact:1,0 ...") and short bench lines (WL)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-q2}; mkdir -p $OUT
if [ -n "$FILES" ]; then
  timeout -k 10 600 python -u -m pytest $FILES ${PYTEST_K:+-k "$PYTEST_K"} -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 11; }
  tail -2 $OUT/pytest.log
fi
for spec in $HOOKAB; do
  IFS=: read w hook vals <<< "$spec"
  AB_REPS=${AB_REPS:-2} timeout -k 10 400 python -u scripts/ab_hook.py $w $hook ${vals//,/ } > $OUT/hook_${w}_${hook}.jsonl 2> $OUT/hook_${w}.err || { tail -20 $OUT/hook_${w}.err; exit 12; }
  echo "hook $w $hook done"
done
for w in $WL; do
  timeout -k 10 300 python -u bench.py --workload $w --steps ${STEPS:-20} --warmup 5 --no-extra --no-cpu-baseline --no-e2e > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 13; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1]); print('$w', d['ms_per_step'], d['value'])"
done
