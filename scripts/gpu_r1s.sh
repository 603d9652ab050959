set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1s
mkdir -p $O
for c in 9 10 11; do
  for dd in 1 2 4; do
    FLTEE_FOLD_CLOG=$c FLTEE_FOLD_DEPTH=$dd timeout -k 10 120 python scripts/fold_ab.py c5 >> $O/fold_ab.jsonl 2>> $O/fold_ab.err || exit 3
  done
done
echo done
