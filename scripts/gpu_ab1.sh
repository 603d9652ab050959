set -o pipefail
mkdir -p gpurun_out/ab1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bitonic or advanced or nips19 or shuffle or sort or pad_skip" > gpurun_out/ab1/pytest.log 2>&1 || exit 11
tail -2 gpurun_out/ab1/pytest.log
L=fl-tee_amd/lib/ab
for w in c5 c4 c3; do
  AB_REPS=2 timeout -k 10 600 python -u scripts/ab_env.py $w FLTEE_LIB=$L/libfltee_agg_ce0lds1.so FLTEE_LIB=$L/libfltee_agg_ce1lds1.so FLTEE_LIB=$L/libfltee_agg_ce1lds2.so FLTEE_LIB=$L/libfltee_agg_ce0lds0.so FLTEE_LIB=$L/libfltee_agg_ce1lds0.so > gpurun_out/ab1/$w.jsonl 2> gpurun_out/ab1/$w.err || exit 12
  echo "ab $w done"
done
