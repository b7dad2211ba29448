# build exp/<NAME>/libairscmp.so from the working tree with extra hipcc flags:
#   build_exp.sh NAME "FLAGS"     (-DAIRS_EXP_ONLY: only the benchmark kernels, faster to build)
set -e
n=$1; f=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/exp/$n"
cd "$ROOT/airs-compression_amd"
make -s build/cmp_host.o build/cmp_gather.o build/decode.o
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $f -I../include -Icsrc"
$H -c csrc/encode.hip -o ../exp/$n/encode.o &
$H -c csrc/enc_stream.hip -o ../exp/$n/enc_stream.o &
$H -c csrc/enc_rice.hip -o ../exp/$n/enc_rice.o &
$H -c csrc/enc_walk.hip -o ../exp/$n/enc_walk.o &
wait
/opt/rocm/bin/hipcc -shared -Wl,-Bsymbolic -Wl,--no-undefined ../exp/$n/encode.o ../exp/$n/enc_rice.o ../exp/$n/enc_stream.o ../exp/$n/enc_walk.o build/decode.o build/cmp_host.o build/cmp_gather.o -ldl -o ../exp/$n/libairscmp.so
rm -f ../exp/$n/encode.o ../exp/$n/enc_rice.o ../exp/$n/enc_stream.o ../exp/$n/enc_walk.o
