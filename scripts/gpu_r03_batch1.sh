# Round-3 batch: persistent A/B (cfg2, cfg4), SALU checksum A/B, then the walk
# kernel's parity tests, the drop-in test and the cfg5 bench + kernel trace.
O=gpurun_out/r03_b1
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
VARIANTS="base pers" WLS="cfg2 cfg4" REPS=2 bash scripts/gpu_ab.sh r03_b1/pers > /dev/null 2>&1 || { echo "pers A/B failed"; cat gpurun_out/r03_b1/pers/ab.jsonl; exit 1; }
cat $O/pers/ab.jsonl
for v in base cksalu; do
  for w in cfg2 cfg4; do
    AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 120 python3 scripts/ck_bench.py $w >> $O/ck.jsonl 2>> $O/ck.err || { echo "ck $v $w failed"; tail -5 $O/ck.err; exit 1; }
  done
done
cat $O/ck.jsonl
AIRS_LIB=exp/cksalu/libairscmp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_checksum.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_ck_salu.log 2>&1; tail -3 $O/pytest_ck_salu.log
bash scripts/gpu_walk_check.sh r03_b1/walk
