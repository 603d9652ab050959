set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_lds
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_lds/a -o run -- python3 scripts/bench_sort.py --sizes 24 --modes 0 --reps 2 > gpurun_out/pmc_lds/a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_lds/b -o run -- python3 scripts/bench_sort.py --sizes 24 --modes 0 --reps 2 > gpurun_out/pmc_lds/b.log 2>&1 || exit 2
echo done
