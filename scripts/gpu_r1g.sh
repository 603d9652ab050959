set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --workload c3 --steps 50 --warmup 5 --no-extra --no-cpu-baseline --no-e2e > $O/c3.json 2> $O/c3.err || exit 4
echo done
