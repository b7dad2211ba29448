# Round 5: sliced Rice selection experiments (timing only: hm1 = no atomics, hm2 = per-wave rows)
TAG=${1:-r05ae}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for L in head new nb4 nb8; do
  case $L in new) unset AIRS_LIB;; *) export AIRS_LIB=exp/$L/libairscmp.so;; esac
  AIRS_KB_AUTO=1 AIRS_KB_ROT=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$L -o kt -- python3 scripts/kbench.py cfg2 > $O/kt_$L.log 2>&1 || { tail $O/kt_$L.log; exit 1; }
  python3 - $O/kt_$L/kt_kernel_stats.csv $L <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'select_rice' in r['Name'] or 'encode_kernel' in r['Name']:
        print(sys.argv[2], r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1000, 2))
PY
done
find $O -name "*.db" -delete
