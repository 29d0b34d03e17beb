#!/bin/bash
# Build the working tree's libhrf.so with extra compile flags into ab/libhrf_<tag>.so (HRF_LIB
# selects it).  usage: bash tools/build_variant.sh <tag> <hipcc flags...>
set -e
tag=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
wt=/tmp/hrf_var_$tag
rm -rf $wt && mkdir -p $wt
cp -r $root/include $wt/ && mkdir -p $wt/hiprfish_image_analysis_amd && cp -r $root/hiprfish_image_analysis_amd/csrc $root/hiprfish_image_analysis_amd/_build.py $root/hiprfish_image_analysis_amd/__init__.py $wt/hiprfish_image_analysis_amd/
(cd $wt && HRF_EXTRA_CFLAGS="$*" python3 -c "from hiprfish_image_analysis_amd import _build; _build.build(verbose=False)")
mkdir -p $root/ab
cp $wt/hiprfish_image_analysis_amd/libhrf.so $root/ab/libhrf_$tag.so
echo built ab/libhrf_$tag.so with "$*"
