# build exp/<NAME>/libairscmp.so with enc_rice.hip compiled with extra flags,
# the other objects from the product build (make first):
#   build_rice_exp.sh NAME "FLAGS"
set -e
n=$1; f=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/exp/$n"
cd "$ROOT/airs-compression_amd"
make -s lib/libairscmp.so
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $f -I../include -Icsrc -c csrc/enc_rice.hip -o ../exp/$n/enc_rice.o
/opt/rocm/bin/hipcc -shared -Wl,-Bsymbolic -Wl,--no-undefined build/encode.o ../exp/$n/enc_rice.o build/enc_stream.o build/enc_walk.o build/decode.o build/cmp_host.o build/cmp_gather.o -ldl -o ../exp/$n/libairscmp.so
rm -f ../exp/$n/enc_rice.o
