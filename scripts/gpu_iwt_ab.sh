# IWT kernel time of exp variants (rocprofv3 kernel stats of scripts/iwt_bench.py)
O=gpurun_out/iwtab
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && \
for v in ${VARIANTS}; do \
  AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o k -- python3 scripts/iwt_bench.py > $O/$v.log 2>&1 || exit 1; \
done
