#!/bin/bash
# round 5: K3C weight-gradient main loop scheduling variants (micro timing + check vs MIOpen)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5/pcw
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in ${VARIANTS:-main pcws1 pcws2}; do
    if [ "$v" = main ]; then lib=vfdepth_amd/libvfd_hip.so; else lib=variants/libvfd_$v.so; fi
    echo "== $v ($rep)"
    VFD_LIB=$lib timeout -k 10 240 python tools/micro_pcw.py --config ${CONFIG:-2} > gpurun_out/r5/pcw/$v.$rep.txt 2>&1 || { tail -5 gpurun_out/r5/pcw/$v.$rep.txt; exit 1; }
    grep -v amdgpu.ids gpurun_out/r5/pcw/$v.$rep.txt
  done
done
