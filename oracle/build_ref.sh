#!/usr/bin/env bash
# Build the REFERENCE's own Cython passes (neighbor2d.pyx, neighbor.pyx) from
# /root/reference, unmodified, into oracle/_ref/.  Test infrastructure only:
# the products are used by tests/golden/make_golden.py to generate the
# committed golden fixtures and to pin the C restatement in oracle/hrf_oracle.c.
#
# Sources compiled (read in place, never copied into the repo):
#   /root/reference/hiprfish-image-analysis-biofilm/neighbor2d.pyx  (line_profile_2d_v2, :8-64)
#   /root/reference/hiprfish-image-analysis-biofilm/neighbor.pyx    (line_profile_v2 :115-181,
#                                                                    line_profile_memory_efficient_v2 :186-263)
# The four neighbor2d.pyx copies in the reference are byte-identical.
# The shipped cpython-35m .so files are never loaded.
#
# Outputs: oracle/_ref/neighbor2d*.so, oracle/_ref/neighbor*.so (+ generated .c)
# Needs: cython, gcc, numpy headers. Skipped (exit 0) when /root/reference is absent.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF=/root/reference/hiprfish-image-analysis-biofilm
OUT="$HERE/_ref"
if [ ! -d "$REF" ]; then
  echo "build_ref: /root/reference absent; skipping reference build" >&2
  exit 0
fi
mkdir -p "$OUT"
PYINC=$(python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")
NPINC=$(python3 -c "import numpy; print(numpy.get_include())")
SUFFIX=$(python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
for mod in neighbor2d neighbor; do
  if [ ! -f "$OUT/$mod$SUFFIX" ] || [ "$REF/$mod.pyx" -nt "$OUT/$mod$SUFFIX" ]; then
    cython -3 --fast-fail -o "$OUT/$mod.c" "$REF/$mod.pyx" 2> "$OUT/$mod.cython.log" || {
      # the reference predates language_level 3; level 2 gives identical outputs
      cython -2 -o "$OUT/$mod.c" "$REF/$mod.pyx" 2>> "$OUT/$mod.cython.log"; }
    gcc -O2 -shared -fPIC -w -I"$PYINC" -I"$NPINC" -DNPY_NO_DEPRECATED_API=0 \
        -o "$OUT/$mod$SUFFIX" "$OUT/$mod.c"
  fi
done
echo "build_ref: built $(ls "$OUT"/*.so | wc -l) reference extension(s) in $OUT"
