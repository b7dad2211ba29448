# checksum kernels: parity, then checksum-enabled cfg2 / cfg4 with both kernels, rocprof of the new one
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ck && export TMPDIR=/tmp || exit 1
O=gpurun_out/ck
timeout -k 10 600 python -u -m pytest tests/test_gpu_checksum.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for w in cfg2 cfg4; do for s in 0 1 2; do
  AIRS_CK_ALG=$s timeout -k 10 300 python scripts/ck_bench.py $w >> $O/ck.jsonl 2>> $O/ck.err || exit 1
done; done
cat $O/ck.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 scripts/ck_bench.py cfg2 > $O/kt.log 2>&1 || exit 1
grep -h "checksum\|encode_kernel" $O/kt/kt_kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
