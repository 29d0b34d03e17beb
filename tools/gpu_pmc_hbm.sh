#!/bin/bash
# HBM traffic of the streaming kernels (channel_sum, register_assemble, label_sums) under
# tools/time_kernels.py stream: kernel trace + one FETCH_SIZE and one WRITE_SIZE --pmc pass
# (separate runs: gfx950 TCC slot limits).  Summarise with profiles/summarize.py.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_hbm
mkdir -p $out
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- \
  python3 tools/time_kernels.py stream > $out/kt.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o pmc -- \
  python3 tools/time_kernels.py stream > $out/fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o pmc -- \
  python3 tools/time_kernels.py stream > $out/write.log 2>&1 &&
echo pmc done
