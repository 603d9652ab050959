set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fold2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "fold or advanced or nips19 or sharded or network" > $O/pytest.log 2>&1 || exit 2
for w in c3 c4 c5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/prof_$w.log 2>&1 || exit 3
done
echo done
