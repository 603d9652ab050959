set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 1 2; do FLTEE_TILEDBG=$v timeout -k 10 300 python scripts/bench_sort.py --sizes 27 --modes 0 --reps 3 > gpurun_out/tdbg_$v.jsonl 2>&1 || exit 1; done
export TMPDIR=/tmp
for v in 0 1 2; do FLTEE_TILEDBG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tdbg_prof_$v -o run -- python3 scripts/bench_sort.py --sizes 27 --modes 0 --reps 2 > gpurun_out/tdbg_prof_$v.log 2>&1 || exit 2; done
echo done
