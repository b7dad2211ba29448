# A/B: build the committed encode.hip as exp/base and the working tree as exp/new,
# then time both (kbench) on the GPU box.  usage: bash scripts/ab.sh  (run locally, then gpurun scripts/gpu_exp.sh)
set -e
rm -rf exp/base exp/new
mkdir -p exp/base
git show HEAD:airs-compression_amd/csrc/encode.hip > exp/base/encode_head.hip
cp exp/base/encode_head.hip airs-compression_amd/csrc/.encode_head_tmp.hip
bash scripts/build_exp.sh new ""
(cd airs-compression_amd && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc \
   -c csrc/.encode_head_tmp.hip -o ../exp/base/encode.o && \
 /opt/rocm/bin/hipcc -shared -Wl,-Bsymbolic -Wl,--no-undefined ../exp/base/encode.o build/cmp_host.o -o ../exp/base/libairscmp.so)
rm -f airs-compression_amd/csrc/.encode_head_tmp.hip exp/base/encode.o exp/base/encode_head.hip
ls exp/*/libairscmp.so
