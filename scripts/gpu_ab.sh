# Interleaved cold A/B of experiment builds (exp/<V>/libairscmp.so, from
# scripts/build_exp.sh) with scripts/kbench.py; every run also checks the
# frames against the reference digest (bitexact field).
#   VARIANTS="base stal" WLS="cfg2 cfg4" REPS=2 bash scripts/gpu_ab.sh TAG
TAG=${1:-ab}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && : > $O/ab.jsonl || exit 1
for rep in $(seq ${REPS:-2}); do for w in ${WLS:-cfg2}; do for v in ${VARIANTS:-base}; do
  echo -n "{\"variant\": \"$v\", \"rep\": $rep, \"kb\": " >> $O/ab.jsonl
  AIRS_KB_ROT=${ROT:-4} AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 120 python scripts/kbench.py $w > $O/one.json 2>> $O/ab.err || { cat $O/one.json; exit 1; }
  cat $O/one.json | tr -d '\n' >> $O/ab.jsonl; echo "}" >> $O/ab.jsonl
done; done; done
cat $O/ab.jsonl
