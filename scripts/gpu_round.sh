# Round deliverable run on the GPU box: smoke, bench line, rocprofv3 kernel
# trace + stats of the bench command, FETCH_SIZE / WRITE_SIZE passes -> traffic,
# then the GPU test suite.  usage: bash scripts/gpu_round.sh TAG
TAG=${1:-r01}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o bench -- python3 bench.py --no-cpu-baseline > $O/kt.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o pf -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pf.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o pw -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pw.log 2>&1 && \
python3 scripts/traffic.py $O/pf/pf_results.db $O/pw/pw_results.db cfg2 $O/traffic_cfg2.json > $O/traffic.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
