"""The watershed tie path on bench.py's adversarial 512x512 plateau image (bench._watershed_ties):
mean hrf_watershed_ex time and tie statistics.  python tools/time_ws_ties.py"""
import json
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402

print(json.dumps(bench._watershed_ties("cuda")))
