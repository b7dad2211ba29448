# Round 5: parity of the restructured enc_rice, the persistent experiment, then the ablation matrix
TAG=${1:-r05h}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && : > $O/abl.jsonl || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_rice.py tests/test_gpu_walk.py tests/test_gpu_autorice.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
AIRS_LIB=exp/persist4/libairscmp.so timeout -k 10 900 python -u -m pytest tests/test_gpu_rice.py tests/test_gpu_walk.py tests/test_gpu_autorice.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "laplace or outliers" > $O/pytest_p.log 2>&1
rc=$?; tail -2 $O/pytest_p.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for w in cfg2 cfg4; do for lib in exp/old exp/w256x4 exp/persist4; do
  AIRS_LIB=$lib/libairscmp.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w $lib', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
for lib in abl abl4; do for w in cfg2 cfg4; do for m in 0 2 512 514 32768 2048; do
  AIRS_KB_ROT=4 AIRS_LIB=exp/$lib/libairscmp.so AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w > $O/one.json 2>> $O/abl.err || { tail -3 $O/abl.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/one.json')); print('$lib', d['workload'], d['dbg'], round(d['median_ms']*1e3,1), round(d['min_ms']*1e3,1))" | tee -a $O/abl.jsonl
done; done; done
