# skip the last tile's self-prefetch in the bitonic tile passes (ts): parity + A/B
mkdir -p gpurun_out/r05ts
P="python -u -m pytest -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread"
FLTEE_LIB=fl-tee_amd/lib/ab/libfltee_agg_ts.so timeout -k 10 500 $P tests/test_gpu_c5_full.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -k "advanced or compaction or sort or shuffle or nips19 or c5_full_size or distributed" > gpurun_out/r05ts/pytest_ts.log 2>&1 && tail -n 2 gpurun_out/r05ts/pytest_ts.log && TAG=r05ts TESTS=0 BENCH=0 AB="c3 a30 c5 c4" ABV="FLTEE_LIB=fl-tee_amd/lib/ab/libfltee_agg_ts.so" bash scripts/gpu_evidence.sh
