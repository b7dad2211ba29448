# Round 5: IWT passes in the device exact mode; the sliced Rice selection rewritten (per-lane bins, fused pick)
TAG=${1:-r05ab}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_autorice.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u scripts/iwt_exact_bench.py > $O/iwt_exact.json 2> $O/iwt_exact.err; rc=$?; cat $O/iwt_exact.json; [ $rc -eq 0 ] || { tail -5 $O/iwt_exact.err; exit $rc; }
for r in 1 2; do
  for L in head new; do
    if [ $L = head ]; then export AIRS_LIB=exp/head/libairscmp.so; else unset AIRS_LIB; fi
    AIRS_KB_AUTO=1 AIRS_KB_ROT=3 timeout -k 10 120 python3 scripts/kbench.py cfg2 > $O/kb_auto4mi_${L}_$r.log 2>&1 || { tail $O/kb_auto4mi_${L}_$r.log; exit 1; }
    echo "$L $(tail -1 $O/kb_auto4mi_${L}_$r.log)"
  done
done
unset AIRS_LIB
AIRS_KB_AUTO=1 AIRS_KB_ROT=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_auto4mi -o kt -- python3 scripts/kbench.py cfg2 > $O/kt_auto4mi.log 2>&1 || { tail $O/kt_auto4mi.log; exit 1; }
find $O -name "*.db" -delete
