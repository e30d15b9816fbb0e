set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider -x --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest_gpu.log 2>&1; echo "pytest rc=$?"
timeout -k 10 600 python bench.py > gpurun_out/r02b/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r02b/bench.log > gpurun_out/r02b/bench.json
PASSES="A B" bash scripts/prof_counters.sh r02b/ctr_ncol1 || exit $?
AON_F16X3_NCOL=2 PASSES="A B" bash scripts/prof_counters.sh r02b/ctr_ncol2 || exit $?
echo done
