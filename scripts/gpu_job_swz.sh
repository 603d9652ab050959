set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/swz1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "swizzle or bitonic or advanced or nips19 or shuffle or sort or pad_skip" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 11; }
tail -2 $OUT/pytest.log
for w in c5 c4; do
  AB_REPS=3 timeout -k 10 300 python -u scripts/ab_hook.py $w fltee_debug_set_swizzle 1 0 > $OUT/ab_$w.jsonl 2> $OUT/ab_$w.err || { tail -20 $OUT/ab_$w.err; exit 12; }
done
echo done
