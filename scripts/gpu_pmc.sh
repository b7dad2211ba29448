# Two rocprofv3 --pmc passes (SQ issue / wait / LDS counters) per workload on
# the product library, cold inputs (bench.py rotates its buffer sets):
#   bash scripts/gpu_pmc.sh TAG [workloads...]      -> gpurun_out/TAG/pmc_summary.json
# The rocprofv3 databases are summarised on the box and then deleted (size).
TAG=${1:-pmc}; shift
WLS=${@:-cfg2 cfg3 cfg5}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
B="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-warm"
for w in $WLS; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_${w}_1 -o p -- python3 $B --workload $w > $O/pmc_${w}_1.log 2>&1 || { tail -5 $O/pmc_${w}_1.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC -d $O/pmc_${w}_2 -o p -- python3 $B --workload $w > $O/pmc_${w}_2.log 2>&1 || { tail -5 $O/pmc_${w}_2.log; exit 1; }
done
python3 scripts/pmc_summary.py $O > $O/pmc_summary.json 2> $O/pmc_summary.err; cat $O/pmc_summary.json | head -c 6000
find $O -name "*.db" -delete
