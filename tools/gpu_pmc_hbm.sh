#!/bin/bash
# HBM traffic of the timed path's streaming kernels (bench.py HBM_KERNELS: channel_max_multi_pf,
# the pixel-table assembly, the calibrated lasers label sums) under tools/time_kernels.py path:
# kernel trace + one FETCH_SIZE and one WRITE_SIZE --pmc pass (separate runs: gfx950 TCC slot
# limits), and the same two passes over the dense-map calibration run of the label sums (4-byte
# lane reads, a width MI355X_MICROARCH.md leaves uncalibrated).  Summarise with
# python tools/pmc_hbm_summary.py <tag> gpurun_out/pmc_hbm.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_hbm
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- \
  python3 tools/time_kernels.py path > $out/kt.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o pmc -- \
  python3 tools/time_kernels.py path > $out/fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o pmc -- \
  python3 tools/time_kernels.py path > $out/write.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/calfetch -o pmc -- \
  python3 tools/time_kernels.py pathcal > $out/calfetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/calwrite -o pmc -- \
  python3 tools/time_kernels.py pathcal > $out/calwrite.log 2>&1 &&
echo pmc done
