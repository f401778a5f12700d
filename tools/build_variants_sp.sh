# Build A/B variants of libsepvad.so that differ only in spectral.hip compile-time switches.
# usage: bash tools/build_variants_sp.sh name1="-DX=1" ...   -> var/lib_<name>.so
set -e
cd "$(dirname "$0")/.."
make -s -C sep-tfanet-vad_amd/csrc ARCH=gfx950
mkdir -p var
objs=$(ls sep-tfanet-vad_amd/csrc/build/*.o | grep -v '/spectral.o$')
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -disable-promote-alloca-to-lds $flags \
      -c sep-tfanet-vad_amd/csrc/spectral.hip -o var/sp_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/lib_$name.so var/sp_$name.o $objs
  rm -f var/sp_$name.o
done
ls var/
