# gpurun job: kernel traces of one workload set (WL) at HEAD, then optional library A/Bs
# (AB="c3:name1,name2 ...") with scripts/ab_env.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-trace}; mkdir -p $OUT
export TMPDIR=/tmp
for w in $WL; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o run \
      -- python3 bench.py --workload "$w" --steps 10 --warmup 3 --no-extra --no-cpu-baseline \
      --no-e2e > "$OUT/prof_$w.log" 2>&1 || exit 13
  echo "profiled $w"
done
for spec in $AB; do
  w=${spec%%:*}; names=${spec#*:}; args=""
  for v in ${names//,/ }; do args="$args FLTEE_LIB=fl-tee_amd/lib/ab/libfltee_agg_$v.so"; done
  AB_REPS=${AB_REPS:-2} timeout -k 10 600 python -u scripts/ab_env.py $w $args > "$OUT/ab_$w.jsonl" 2> "$OUT/ab_$w.err" || { tail -20 "$OUT/ab_$w.err"; exit 12; }
  echo "ab $w done"
done
