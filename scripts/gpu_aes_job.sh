# gpurun job: AES-CTR parity + A/B of the decrypt kernels (TAG names the output dir)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-aes}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "decrypt" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_aes.log 2>&1 || { tail -30 $OUT/pytest_aes.log; exit 11; }
tail -2 $OUT/pytest_aes.log
timeout -k 10 120 python -u scripts/bench_aes.py > $OUT/ab.jsonl 2>&1 || exit 12
FLTEE_AES_BS=32 timeout -k 10 120 python -u scripts/bench_aes.py >> $OUT/ab.jsonl 2>&1 || exit 13
FLTEE_AES_TTABLE=1 timeout -k 10 120 python -u scripts/bench_aes.py >> $OUT/ab.jsonl 2>&1 || exit 14
grep variant $OUT/ab.jsonl
if [ "${REST:-0}" = 1 ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_client.py tests/test_gpu_ecalls.py tests/test_gpu_server_edges.py tests/test_abi_host.py tests/test_gpu_reference_aggregate.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_rest.log 2>&1 || { tail -30 $OUT/pytest_rest.log; exit 15; }
tail -2 $OUT/pytest_rest.log
fi
