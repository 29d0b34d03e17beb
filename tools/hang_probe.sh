#!/bin/bash
# the six-stream full-size tile test, new component numbering off, then (if that ended without
# a time-out) on
mkdir -p gpurun_out
T=tests/test_tile_gpu.py::test_tile_native_six_streams_fullsize
HRF_LABEL_ONEPASS=0 timeout -k 10 170 python -u -m pytest -x -v --timeout 160 --timeout-method thread $T > gpurun_out/hang0.txt 2>&1
rc=$?
echo "onepass=0 rc=$rc"
tail -5 gpurun_out/hang0.txt
case $rc in 0|1) ;; *) exit 1;; esac
timeout -k 10 170 python -u -m pytest -x -v --timeout 160 --timeout-method thread $T > gpurun_out/hang1.txt 2>&1
rc=$?
echo "onepass=1 rc=$rc"
tail -5 gpurun_out/hang1.txt
