#!/bin/bash
# Round 6: the K3C data gradient's tile order (VFD_PF_NBAND n-tiles per band, variants built by
# tools/build_variant.py): micro timing + parity of each build at config 2.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/pfband
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/micro_projconv.py --config 2 > $OUT/base.log 2>&1 || exit 1
grep "dgrad" $OUT/base.log
for nb in 3 5 25; do
  VFD_LIB=variants/libvfd_pfnb$nb.so timeout -k 10 300 python tools/micro_projconv.py --config 2 > $OUT/nb$nb.log 2>&1 || exit 1
  echo "nband $nb:"; grep "dgrad" $OUT/nb$nb.log
done
