# Round 5: packed-math binning in the sliced Rice selection: autorice tests, A/B against HEAD
TAG=${1:-r05ai}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_autorice.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
bash scripts/gpu_r05_ae.sh $TAG/ae
for r in; do
  for L in head new; do
    if [ $L = head ]; then export AIRS_LIB=exp/head/libairscmp.so; else unset AIRS_LIB; fi
    AIRS_KB_AUTO=1 AIRS_KB_ROT=3 timeout -k 10 120 python3 scripts/kbench.py cfg2 > $O/kb_auto4mi_${L}_$r.log 2>&1 || { tail $O/kb_auto4mi_${L}_$r.log; exit 1; }
    echo "$L $(tail -1 $O/kb_auto4mi_${L}_$r.log)"
  done
done
