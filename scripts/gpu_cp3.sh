set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cp3
mkdir -p $O
export TMPDIR=/tmp
for b in 2 3; do
FLTEE_COMPACT_BLOCKS=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$b -o run -- python3 bench.py --workload c5 --steps 6 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/c5_$b.json 2> $O/c5_$b.err || exit 2
done
FLTEE_COMPACT_BLOCKS=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "advanced" > $O/pytest.log 2>&1 || exit 3
echo done
