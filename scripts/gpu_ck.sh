# checksum-enabled encode: variants (VARIANTS, exp builds) x workloads, rocprofv3 stats
O=gpurun_out/ck
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && \
for v in ${VARIANTS:-prod}; do for w in cfg2 cfg4; do \
  L=$([ $v = prod ] && echo airs-compression_amd/lib/libairscmp.so || echo exp/$v/libairscmp.so); \
  AIRS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$w -o k -- python3 scripts/ck_bench.py $w > $O/${v}_$w.log 2>&1 || exit 1; \
done; done
