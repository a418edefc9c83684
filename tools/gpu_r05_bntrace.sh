#!/bin/bash
# BN UNet b256 kernel traces under knob settings (same box): default, no skip-z, no dual input
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bntrace
R=$PWD; O=gpurun_out/bntrace
prof() {
  local tag=$1; shift
  rm -rf $O/$tag
  (cd /tmp && env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$tag -o run -- python3 $R/bench.py --model unet-bn --steps 5 --warmup 2 > $R/$O/$tag.log 2>&1) || { echo "$tag prof failed"; exit 1; }
  python tools/prof_summary.py $O/$tag > $O/sum_$tag.txt 2>&1
  echo "== $tag: $(grep 'total kernel time' $O/sum_$tag.txt) | $(grep 'last step' $O/sum_$tag.txt | cut -c1-60)"
}
prof base DPA_X=0
prof noskipz DPA_NO_BN_SKIP_Z=1
prof nodual DPA_NO_BN_DUAL=1
prof nohalves DPA_NO_BN_HALVES=1
