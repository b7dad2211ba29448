# build exp/<NAME>/libairscmp.so with extra hipcc flags: build_exp.sh NAME "FLAGS"
set -e
n=$1; f=$2
mkdir -p exp/$n
cd airs-compression_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $f -I../include -Icsrc -c csrc/encode.hip -o ../exp/$n/encode.o
/opt/rocm/bin/hipcc -shared -Wl,-Bsymbolic -Wl,--no-undefined ../exp/$n/encode.o build/cmp_host.o -o ../exp/$n/libairscmp.so
rm -f ../exp/$n/encode.o
