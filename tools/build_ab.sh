#!/bin/bash
# Build libhrf.so of a git revision into ab/libhrf_<tag>.so for interleaved A/B runs
# (HRF_LIB=ab/libhrf_<tag>.so selects it).  usage: bash tools/build_ab.sh <rev> <tag>
set -e
rev=$1; tag=$2
root=$(cd "$(dirname "$0")/.." && pwd)
wt=/tmp/hrf_ab_$tag
rm -rf $wt
git -C $root worktree add --detach $wt $rev > /dev/null
(cd $wt && python3 -c "from hiprfish_image_analysis_amd import _build; _build.build(verbose=False)")
mkdir -p $root/ab
cp $wt/hiprfish_image_analysis_amd/libhrf.so $root/ab/libhrf_$tag.so
git -C $root worktree remove --force $wt
echo built ab/libhrf_$tag.so from $rev
