# checksum kernels: parity, then checksum-enabled cfg2 / cfg4 per kernel (overlapped with the encode, and not), rocprof
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ck && export TMPDIR=/tmp || exit 1
O=gpurun_out/ck
timeout -k 10 600 python -u -m pytest tests/test_gpu_checksum.py tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for w in cfg2 cfg4; do for s in 0 1; do
  AIRS_CK_ALG=$s timeout -k 10 300 python scripts/ck_bench.py $w >> $O/ck.jsonl 2>> $O/ck.err || exit 1
done
  AIRS_CK_OVERLAP=0 timeout -k 10 300 python scripts/ck_bench.py $w | sed 's/}$/, "overlap": 0}/' >> $O/ck.jsonl 2>> $O/ck.err || exit 1
done
cat $O/ck.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 scripts/ck_bench.py cfg2 > $O/kt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o kt -- python3 scripts/ck_bench.py cfg4 > $O/kt4.log 2>&1 || exit 1
