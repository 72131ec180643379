cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in base nogather; do
  if [ $v = base ]; then L=vfdepth_amd/libvfd_hip.so; else L=variants/libvfd_$v.so; fi
  echo "== $v" >> gpurun_out/pcvar.log
  VFD_LIB=$L timeout -k 10 120 python tools/micro_projconv.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/pcvar.log || exit 1
done
