# Sliced Rice selection: GPU suite on the product library, then cfg2-shaped
# AUTO_RICE calls (16 x 4 Mi, the sliced path) with the old (exp/sel0) and new
# (exp/sel1) library, cold.   bash scripts/gpu_sel_ab.sh TAG
TAG=${1:-sel}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && : > $O/ab.jsonl || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in sel0 sel1; do
  AIRS_KB_AUTO=1 AIRS_KB_ROT=4 AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 120 python scripts/kbench.py cfg2 > $O/one.json 2>> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/one.json')); d['variant']='$v'; d['rep']=$rep; print(json.dumps(d))" >> $O/ab.jsonl
done; done
cat $O/ab.jsonl
