set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_pmc.sh r1c 2 > gpurun_out/pmc_r1c.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bench_kt -o kt -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/bench_kt.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/bench_r1c.json 2> gpurun_out/bench_r1c.err &&
echo all done
