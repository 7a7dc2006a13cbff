# round 5: the whole GPU suite on HEAD, smoke, then the default bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ -s > gpurun_out/r5_gpu_tests.log 2>&1
echo "tests rc=$?"
tail -3 gpurun_out/r5_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r5_bench.log 2>&1
echo "bench rc=$?"
