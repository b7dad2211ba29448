# Round 5: LDS bank-conflict ablation of the Rice kernel (exp/abl, -DAIRS_ABLATE=1):
# per mode the cold kernel time (kbench) and one PMC pass (LDS instructions, conflict cycles, VALU)
TAG=${1:-r05r}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && : > $O/abl.jsonl || exit 1
for w in cfg2 cfg4; do for m in 0 4096 32 2048 6176; do
  AIRS_KB_ROT=4 AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w > $O/one.json 2>> $O/abl.err || { tail -3 $O/abl.err; exit 1; }
  AIRS_KB_ROT=4 AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=$m timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/p_${w}_$m -o p -- python3 scripts/kbench.py $w > $O/p_${w}_$m.log 2>&1 || { tail -3 $O/p_${w}_$m.log; exit 1; }
  python3 - $O/one.json $O/p_${w}_$m $w $m >> $O/abl.jsonl <<'PY'
import glob, json, sys
sys.path.insert(0, "scripts")
import rocpd_summary
one = json.load(open(sys.argv[1]))
cnt = {}
for db in glob.glob(sys.argv[2] + "/**/*.db", recursive=True):
    ks, c = rocpd_summary.summarise(db, "rice_kernel")
    for (kn, cn), v in c.items():
        cnt[cn] = v
r = dict(workload=sys.argv[3], dbg=int(sys.argv[4]), median_us=round(one["median_ms"] * 1e3, 1),
         min_us=round(one["min_ms"] * 1e3, 1), **cnt)
if cnt.get("SQ_INSTS_LDS"):
    r["conflict_cycles_per_lds_inst"] = round(cnt.get("SQ_LDS_BANK_CONFLICT", 0) / cnt["SQ_INSTS_LDS"], 3)
if cnt.get("GRBM_GUI_ACTIVE") and cnt.get("SQ_ACTIVE_INST_VALU"):
    r["valu_busy"] = round(cnt["SQ_ACTIVE_INST_VALU"] * 4 / (cnt["GRBM_GUI_ACTIVE"] / 8 * 1024), 3)
print(json.dumps(r))
PY
  tail -1 $O/abl.jsonl | cut -c1-400
done; done
find $O -name "*.db" -delete
