#!/bin/bash
# Round 6: the half-width groups' bias in the K3C data gradient's group split (VFD_PF_HBIAS
# variants by tools/build_variant.py): C-ABI micro timing at config 2, default build first.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/pfhbias
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/micro_projconv.py --config 2 > $OUT/b1.log 2>&1 || exit 1
echo "bias 1:"; grep folded $OUT/b1.log
for b in 0 2 4; do
  VFD_LIB=variants/libvfd_pfh$b.so timeout -k 10 300 python tools/micro_projconv.py --config 2 > $OUT/b$b.log 2>&1 || exit 1
  echo "bias $b:"; grep folded $OUT/b$b.log
done
timeout -k 10 300 python tools/micro_projconv.py --config 2 > $OUT/b1_again.log 2>&1 || exit 1
echo "bias 1 again:"; grep folded $OUT/b1_again.log
