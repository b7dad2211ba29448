# kernel trace of one experiment build on one workload: AIRS_LIB=exp/V ... bash scripts/gpu_r03_kt.sh TAG V W
O=gpurun_out/$1
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
AIRS_LIB=exp/$2/libairscmp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --workload $3 --no-cpu-baseline --no-warm > $O/kt.json 2> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" | xargs cat | cut -c1-160 | head -6
python3 -c "import json; d=json.load(open('$O/kt.json')); print('$3', d['ms_per_step'], d['roofline']['avg_launch_ms_hip_events'])"
