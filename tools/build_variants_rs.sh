# Build A/B variants of libsepvad.so that differ only in tcn_rs.hip compile-time switches.
# usage: bash tools/build_variants_rs.sh name1="-DRS_X=1" ...   -> var/lib_<name>.so
set -e
cd "$(dirname "$0")/.."
make -s -C sep-tfanet-vad_amd/csrc ARCH=gfx950
mkdir -p var
objs=$(ls sep-tfanet-vad_amd/csrc/build/*.o | grep -v '/tcn_rs.o$')
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-variable -mllvm -disable-promote-alloca-to-lds \
      -fno-slp-vectorize $flags -c sep-tfanet-vad_amd/csrc/tcn_rs.hip -o var/tcn_rs_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/lib_$name.so var/tcn_rs_$name.o $objs \
      -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
  rm -f var/tcn_rs_$name.o
done
