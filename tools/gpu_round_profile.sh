set -o pipefail
mkdir -p gpurun_out/r2a
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 420 python -u bench.py > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2a/prof -o run -- python3 bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/r2a/prof_bench.json 2> gpurun_out/r2a/prof.err
