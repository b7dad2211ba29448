# Round 5: FETCH_SIZE of the sliced Rice selection kernel, HEAD vs working tree vs no-atomics build
TAG=${1:-r05af}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for L in head new hm1; do
  case $L in new) unset AIRS_LIB;; *) export AIRS_LIB=exp/$L/libairscmp.so;; esac
  AIRS_KB_AUTO=1 AIRS_KB_ROT=3 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum -d $O/pmc_$L -o p -- python3 scripts/kbench.py cfg2 > $O/pmc_$L.log 2>&1 || { tail -5 $O/pmc_$L.log; exit 1; }
  python3 scripts/rocpd_summary.py $(find $O/pmc_$L -name "*.db") --kernel select_rice_hist > $O/pmc_$L.txt 2>&1; grep -v "^==" $O/pmc_$L.txt | cut -c1-160
done
find $O -name "*.db" -delete
