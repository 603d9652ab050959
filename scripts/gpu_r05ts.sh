# HEAD validation: full GPU tests, bench, smoke
TAG=r05z5 TESTS=1 BENCH=1 bash scripts/gpu_evidence.sh || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z5/smoke.log 2>&1 || exit 1
tail -n 1 gpurun_out/r05z5/smoke.log
