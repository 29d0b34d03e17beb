#!/bin/bash
# Round profile: GPU suite, the full bench line, the kernel-trace stats of the same bench
# command, classifier PMC passes, the streaming kernels' PMC passes.
# usage: bash tools/gpu_round.sh <tag> [notest]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r4}
o=gpurun_out/$tag
mkdir -p $o
if [ "$2" != "notest" ]; then
# no -x: a failing parity test is reported and the measurements still run (a fault or a hang
# -- exit status 124/134/137/139 -- ends the call)
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $o/pytest_gpu.txt 2>&1
rc=$?
tail -3 $o/pytest_gpu.txt
case $rc in 0|1) ;; *) echo "test run ended with status $rc"; exit 1;; esac
fi
timeout -k 10 600 python -u bench.py > $o/bench.json 2> $o/bench.err || { echo "bench failed"; tail -30 $o/bench.err; exit 1; }
cut -c1-300 $o/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline > $o/prof_bench.json 2> $o/prof.err || { echo "profile failed"; exit 1; }
bash tools/gpu_pmc.sh $tag t || { echo "pmc failed"; exit 1; }
bash tools/gpu_pmc_hbm.sh || { echo "pmc hbm failed"; exit 1; }
bash tools/gpu_pmc_nlm.sh $tag || { echo "pmc nlm failed"; exit 1; }
echo round done
