# Round 4: diagnostic of the walk fallback, GPU suite (all tests, no -x), env/lib A/B, bench lines.
TAG=${1:-r04b}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 250 python exp/diag_walkfb.py u16 > $O/diag.log 2>&1; rc=$?
tail -30 $O/diag.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > $O/ab.jsonl
for rep in 1 2; do for w in ${WLS:-cfg2}; do for v in ${VARIANTS:-base}; do
  name=${v%%:*}; envs=""; [ "$name" != "$v" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
  echo -n "{\"variant\": \"$name\", \"rep\": $rep, \"kb\": " >> $O/ab.jsonl
  env $envs AIRS_KB_ROT=4 timeout -k 10 120 python scripts/kbench.py $w > $O/one.json 2>> $O/ab.err || { cat $O/one.json; tail -5 $O/ab.err; exit 1; }
  cat $O/one.json | tr -d '\n' >> $O/ab.jsonl; echo "}" >> $O/ab.jsonl
done; done; done
cut -c1-220 $O/ab.jsonl
for w in ${BENCH_WLS:-}; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['value'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'], r.get('frac_samples_only'))"
done
