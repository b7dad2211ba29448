# build exp/<NAME>/libairscmp.so with the decoder compiled with extra flags:
#   build_dec_exp.sh NAME "FLAGS"
set -e
n=$1; f=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/exp/$n"
cd "$ROOT/airs-compression_amd"
make -s build/cmp_host.o build/encode.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $f -I../include -Icsrc -c csrc/decode.hip -o ../exp/$n/decode.o
/opt/rocm/bin/hipcc -shared -Wl,-Bsymbolic -Wl,--no-undefined build/encode.o ../exp/$n/decode.o build/cmp_host.o -o ../exp/$n/libairscmp.so
rm -f ../exp/$n/decode.o
