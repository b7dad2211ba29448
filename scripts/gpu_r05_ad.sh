# Round 5: PMC pass on the sliced Rice selection kernel (HEAD vs working tree)
TAG=${1:-r05ad}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for L in head new; do
  if [ $L = head ]; then export AIRS_LIB=exp/head/libairscmp.so; else unset AIRS_LIB; fi
  AIRS_KB_AUTO=1 AIRS_KB_ROT=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT -d $O/pmc_$L -o p -- python3 scripts/kbench.py cfg2 > $O/pmc_$L.log 2>&1 || { tail -5 $O/pmc_$L.log; exit 1; }
  python3 scripts/rocpd_summary.py $(find $O/pmc_$L -name "*.db") --kernel select_rice > $O/pmc_$L.txt 2>&1; cat $O/pmc_$L.txt | head -30
done
find $O -name "*.db" -delete
