set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final_${TAG:-x}
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_${TAG:-x}/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/final_${TAG:-x}/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/final_${TAG:-x}/pytest_gpu.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 900 python bench.py > gpurun_out/final_${TAG:-x}/bench.json 2> gpurun_out/final_${TAG:-x}/bench.err || exit 3
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_${TAG:-x}/prof_ns -o run -- python3 bench.py --steps 25 --no-extra --no-cpu-baseline --no-e2e > gpurun_out/final_${TAG:-x}/prof_ns.log 2>&1 || exit 4
echo done
