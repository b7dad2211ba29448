# host-API probe on a plain C process, the host-API parity tests, then the
# PMC passes of cfg5 (walk kernel) and cfg2
O=gpurun_out/r03_b3
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 60 tests/dropin/host_probe > $O/probe.out 2> $O/probe.err; echo "probe rc=$?"; cat $O/probe.out; tail -c 3000 $O/probe.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.log 2>&1; rc=$?
tail -5 $O/pytest_parity.log | cut -c1-300
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_pmc.sh r03_b3/pmc cfg5 cfg2 > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
python3 -c "
import json; d=json.load(open('$O/pmc/pmc_summary.json'))
for w,v in d.items(): print(w, json.dumps(v.get('_per_sample_dominant')))
"
