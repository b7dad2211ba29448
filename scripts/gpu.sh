# The one GPU-box runner: named steps, each under its own time limit, chained
# so that the first failure ends the call.  Output under gpurun_out/TAG.
#   gpurun --timeout 900 -- bash scripts/gpu.sh TAG STEP [STEP ...]
# steps:
#   tests            the whole -m gpu suite, then smoke()
#   tests:EXPR       the -m gpu tests selected by -k EXPR
#   bench:W          bench.py --workload W (cfg2 with the CPU baseline)
#   kt:W             rocprofv3 kernel trace + stats of bench.py --workload W
#   traffic:W        FETCH_SIZE and WRITE_SIZE passes (separate runs) -> traffic_W.json
#   pmcsum:W         the two SQ counter passes over bench.py W -> pmc_summary.json (scripts/pmc_summary.py)
#   pmc:W:C1,C2,...  one PMC pass (counters within one pass's limits) over kbench W
#   kb:W[:LIB]       scripts/kbench.py W, cold (3 rotated sets), exp/LIB/libairscmp.so if given
#   kbt:W[:LIB]      kb:W under a rocprofv3 kernel trace (110 launches, per-launch durations)
#   ts:W:LIB         the per-segment timeline ring of 110 cold launches (ablation build LIB,
#                    AIRS_DBG 65536, or $AIRS_DBG) under a kernel trace; scripts/ts_launches.py reads it
#   run:NAME         exp/bin/NAME (a micro-benchmark built from scripts/NAME.hip)
#   env:VAR=VALUE    export VAR for the following steps;  unset:VAR  drop it again
# kb, kbt and ts take an optional 4th field, a tag appended to their output names.
# Environment variables set before the command (AIRS_*) reach every step.
TAG=$1
shift
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
kern() {
	case $1 in
	cfg2 | cfg2s | cfg3 | cfg4) echo rice_kernel ;;
	cfg5 | cfg5fb) echo walk_ctx_kernel ;;
	cfg5s8 | cfg5fbs8) echo walk_kernel ;;
	esac
}
libenv() { [ -n "$1" ] && echo "AIRS_LIB=exp/$1/libairscmp.so"; }
for st in "$@"; do
	IFS=: read -r what w x tg <<<"$st"
	echo "== $st"
	case $what in
	tests)
		sel=()
		[ -n "$w" ] && sel=(-k "$w")
		timeout -k 10 900 python -u -m pytest tests -m gpu -x -q "${sel[@]}" --timeout 300 --timeout-method thread \
			-p no:cacheprovider >$O/pytest_gpu.log 2>&1
		rc=$?
		tail -3 $O/pytest_gpu.log | cut -c1-200
		[ $rc -eq 0 ] || { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; exit $rc; }
		if [ -z "$w" ]; then
			timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >$O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
			tail -1 $O/smoke.log
		fi
		;;
	bench)
		cpu=--no-cpu-baseline
		[ "$w" = cfg2 ] && cpu=
		timeout -k 10 400 python bench.py --workload $w $cpu >$O/bench_$w.json 2>$O/bench_$w.err || { tail $O/bench_$w.err; exit 1; }
		python3 -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['value'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'], r.get('launch_us'))"
		;;
	kt)
		timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$w -o kt -- python3 bench.py \
			--workload $w --no-cpu-baseline --no-warm >$O/kt_$w.log 2>&1 || { tail $O/kt_$w.log; exit 1; }
		python3 scripts/launch_stats.py $O/kt_$w/kt_kernel_trace.csv $(kern $w)
		# the 25 launches after bench.py's 5 untimed warmups (its 20 timed steps
		# and the first 5 of its separate per-launch pass)
		python3 scripts/launch_stats.py $O/kt_$w/kt_kernel_trace.csv $(kern $w) --skip 5 --count 25 \
			--json $O/kt_${w}_launches.json
		;;
	traffic)
		K=$(kern $w)
		timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$w -o pf -- python3 bench.py --workload $w --steps 5 \
			--warmup 1 --no-cpu-baseline --no-warm >$O/pf_$w.log 2>&1 || { tail -3 $O/pf_$w.log; exit 1; }
		timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pw_$w -o pw -- python3 bench.py --workload $w --steps 5 \
			--warmup 1 --no-cpu-baseline --no-warm >$O/pw_$w.log 2>&1 || { tail -3 $O/pw_$w.log; exit 1; }
		python3 scripts/traffic.py $O/pf_$w/pf_results.db $O/pw_$w/pw_results.db $w $O/traffic_$w.json --kernel $K \
			>$O/traffic_$w.log 2>&1 || { tail -3 $O/traffic_$w.log; exit 1; }
		cut -c1-300 $O/traffic_$w.json
		find $O -name "*.db" -delete
		;;
	pmcsum)
		# the two SQ passes of the encode kernels on bench.py --workload W -> pmc_summary.json
		B="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-warm --workload $w"
		timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
			SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_${w}_1 -o p -- \
			python3 $B >$O/pmc_${w}_1.log 2>&1 || { tail -5 $O/pmc_${w}_1.log; exit 1; }
		timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
			SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC -d $O/pmc_${w}_2 -o p -- \
			python3 $B >$O/pmc_${w}_2.log 2>&1 || { tail -5 $O/pmc_${w}_2.log; exit 1; }
		python3 scripts/pmc_summary.py $O >$O/pmc_summary_$w.json 2>$O/pmc_summary.err
		python3 -c "import json; d=json.load(open('$O/pmc_summary_$w.json')); print(json.dumps({k: v.get('_per_sample_dominant') for k, v in d.items()})[:1500])"
		find $O -name "*.db" -delete
		;;
	pmc)
		tagp=$(echo "$x" | tr ',' '_' | cut -c1-40)_d${AIRS_DBG:-0}
		AIRS_KB_ROT=3 timeout -s KILL 90 rocprofv3 --pmc ${x//,/ } --output-format csv \
			-d $O/pmc_${w}_$tagp -o p -- python3 scripts/kbench.py $w >$O/pmc_${w}_$tagp.log 2>&1 || { tail -3 $O/pmc_${w}_$tagp.log; exit 1; }
		;;
	kb)
		# kb:W[:LIB[:DBG]]  (DBG: AIRS_DBG ablation bits, ablation builds only)
		env $(libenv "$x") ${tg:+AIRS_DBG=$tg} AIRS_KB_ROT=3 timeout -k 10 120 python scripts/kbench.py $w >>$O/kb.jsonl 2>>$O/kb.err || { tail -3 $O/kb.err; exit 1; }
		tail -1 $O/kb.jsonl
		;;
	kbt)
		d=$O/kbt_${w}_${x:-prod}${tg:+_$tg}
		env $(libenv "$x") AIRS_KB_ROT=3 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- \
			python3 scripts/kbench.py $w >$d.log 2>&1 || { tail -3 $d.log; exit 1; }
		tail -1 $d.log
		python3 scripts/launch_stats.py $d/kt_kernel_trace.csv $(kern $w)
		;;
	ts)
		d=$O/ts_${w}_$x${tg:+_$tg}
		env $(libenv "$x") AIRS_KB_ROT=3 AIRS_DBG=${AIRS_DBG:-65536} AIRS_DBGTS_RING=$((110 + ${AIRS_KB_PRE:-0})) \
			AIRS_DBGTS_PATH=$d.bin timeout -k 10 200 \
			rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 scripts/kbench.py $w >$d.log 2>&1 || { tail -3 $d.log; exit 1; }
		tail -1 $d.log
		python3 scripts/launch_stats.py $d/kt_kernel_trace.csv $(kern $w)
		spf=256
		[ "$w" = cfg4 ] && spf=4
		if [ "$w" = cfg3 ]; then
			python3 scripts/ts_auto.py $d.bin $((110 + ${AIRS_KB_PRE:-0})) >$d.txt 2>&1
		else
			python3 scripts/ts_launches.py $d.bin $((110 + ${AIRS_KB_PRE:-0})) $spf >$d.txt 2>&1
		fi
		head -12 $d.txt
		gzip $d.bin
		;;
	run)
		# run:NAME  a prebuilt exp/bin/NAME (scripts/*.hip micro-benchmarks)
		timeout -k 10 120 exp/bin/$w >$O/run_$w.txt 2>&1 || { tail -5 $O/run_$w.txt; exit 1; }
		cat $O/run_$w.txt
		;;
	env)
		export "$w${x:+:$x}"
		;;
	unset)
		unset "$w"
		;;
	*)
		echo "unknown step $st"
		exit 2
		;;
	esac
done
exit 0
