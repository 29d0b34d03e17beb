set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/it7
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/it7/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/it7/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/it7/pytest_gpu.txt
timeout -k 10 120 python -u tools/time_kernels.py nlmeans 2>&1 | grep nl_means
AB_REPS=3 timeout -k 10 700 bash tools/bench_ab.sh HRF_PRIORITY=1 HRF_PRIORITY=2 && cat gpurun_out/ab.log
