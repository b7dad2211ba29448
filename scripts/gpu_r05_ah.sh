# Round 5: one-launch IWT batches (asynchronous mode): batch tests + IWT timings
TAG=${1:-r05ah}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u scripts/iwt_exact_bench.py > $O/iwt_exact.json 2> $O/iwt_exact.err; rc=$?; cat $O/iwt_exact.json; [ $rc -eq 0 ] || { tail -5 $O/iwt_exact.err; exit $rc; }
