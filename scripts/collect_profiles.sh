# Copy a round's GPU evidence from gpurun_out/ into profiles/ (tracked):
#   collect_profiles.sh RUN_TAG PROF_TAG PMC_TAG PREFIX
# RUN_TAG: a scripts/gpu.sh run with tests and bench:W steps;
# PROF_TAG: one with kt:W and traffic:W steps (kernel stats, FETCH/WRITE traffic);
# PMC_TAG: one with pmc:W:... steps (scripts/pmc_summary.py -> pmc_summary.json).  Missing pieces are skipped.
R=gpurun_out/$1; P=gpurun_out/$2; M=gpurun_out/$3; X=profiles/$4
for f in $R/bench_*.json; do [ -f "$f" ] && cp "$f" ${X}_$(basename "$f"); done
[ -f $R/pytest_gpu.log ] && tail -5 $R/pytest_gpu.log > ${X}_pytest_gpu.txt
[ -f $R/smoke.log ] && cp $R/smoke.log ${X}_smoke.txt
for d in $P/kt_*/; do
  [ -d "$d" ] || continue
  w=$(basename "$d"); w=${w#kt_}
  [ -f "$d/kt_kernel_stats.csv" ] && cp "$d/kt_kernel_stats.csv" ${X}_kernel_stats_$w.csv
done
for f in $P/traffic_*.json; do [ -f "$f" ] && cp "$f" ${X}_$(basename "$f"); done
[ -f $M/pmc_summary.json ] && cp $M/pmc_summary.json ${X}_pmc_summary.json
ls ${X}_* | wc -l
