set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 2
for c in 0 11 12 13; do
  for dd in 0 2 4; do
    FLTEE_FOLD_CLOG=$c FLTEE_FOLD_DEPTH=$dd timeout -k 10 120 python scripts/fold_ab.py c5 >> $O/fold_ab.jsonl 2>> $O/fold_ab.err || exit 3
  done
done
for w in c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/prof_$w.log 2>&1 || exit 4
done
echo done
