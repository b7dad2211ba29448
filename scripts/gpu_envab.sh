# Interleaved cold A/B of environment variants of ONE library build with
# scripts/kbench.py; every run also checks the frames against the reference
# digest (bitexact field).  A variant is NAME or NAME:VAR=VAL,VAR=VAL.
#   VARIANTS="old:AIRS_ARENA=0 new:AIRS_ARENA=1" WLS="cfg2 cfg4" REPS=2 bash scripts/gpu_envab.sh TAG
TAG=${1:-envab}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && : > $O/ab.jsonl || exit 1
for rep in $(seq ${REPS:-2}); do for w in ${WLS:-cfg2}; do for v in ${VARIANTS:-base}; do
  name=${v%%:*}; envs=""; [ "$name" != "$v" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
  echo -n "{\"variant\": \"$name\", \"rep\": $rep, \"kb\": " >> $O/ab.jsonl
  env $envs AIRS_KB_ROT=${ROT:-4} timeout -k 10 120 python scripts/kbench.py $w > $O/one.json 2>> $O/ab.err || { cat $O/one.json; tail -5 $O/ab.err; exit 1; }
  cat $O/one.json | tr -d '\n' >> $O/ab.jsonl; echo "}" >> $O/ab.jsonl
done; done; done
cat $O/ab.jsonl
