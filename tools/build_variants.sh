# Build A/B variants of libsepvad.so that differ only in compile-time switches of the fused TCN (tcn_kernel.h) for the
# production combination (fp16x3, int8 lo plane: build/fused_x3l2.o); every other object is the tree's own.
# usage: bash tools/build_variants.sh name1="-DTCN_X=0" name2="-DTCN_Y=0 -DTCN_Z=0" ...   -> abl/lib_<name>.so
# VARIANT_L0=1: the fp16-lo object too (build/fused_x3l0.o: the two-slice launches stream the int8 values as fp16, api.hip twfq)
set -e
cd "$(dirname "$0")/.."
make -s -C sep-tfanet-vad_amd/csrc ARCH=gfx950
mkdir -p abl
if [ -n "$VARIANT_L0" ]; then
  objs=$(ls sep-tfanet-vad_amd/csrc/build/*.o | grep -v '/fused_x3l2.o$' | grep -v '/fused_x3l0.o$')
else
  objs=$(ls sep-tfanet-vad_amd/csrc/build/*.o | grep -v '/fused_x3l2.o$')
fi
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-variable -mllvm -disable-promote-alloca-to-lds $flags \
      -DFI_PRE=PREC_F16X3 -DFI_LQ=2 -c sep-tfanet-vad_amd/csrc/fused_inst.hip -o abl/fused_$name.o &
  if [ -n "$VARIANT_L0" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-variable -mllvm -disable-promote-alloca-to-lds $flags \
        -DFI_PRE=PREC_F16X3 -DFI_LQ=0 -c sep-tfanet-vad_amd/csrc/fused_inst.hip -o abl/fused0_$name.o &
  fi
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  l0=""; [ -n "$VARIANT_L0" ] && l0=abl/fused0_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/lib_$name.so abl/fused_$name.o $l0 $objs \
      -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
  rm -f abl/fused_$name.o abl/fused0_$name.o
done
ls -la abl/
