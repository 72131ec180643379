#!/bin/bash
# Round 5: one-launch channels-last BN for the depth encoder's small layers (VFD_BN1_NHWC=1 build)
# with the branch streams: BN tests on the variant, then bench A/B alternating
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/jj
mkdir -p $OUT
export PYTHONUNBUFFERED=1
VFD_LIB=variants/libvfd_bn1n.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "batchnorm or channels_last" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || exit $rc
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
pr() { python -c "import json;d=json.load(open('$OUT/$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
  VFD_LIB=variants/libvfd_bn1n.so timeout -k 10 300 python bench.py $B > $OUT/one$i.json 2> $OUT/one$i.err && pr one$i || exit 1
  timeout -k 10 300 python bench.py $B > $OUT/base$i.json 2> $OUT/base$i.err && pr base$i || exit 1
done
