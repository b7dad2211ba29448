# look-back statistics (AIRS_DBG=256) of exp variants built with -DAIRS_ABLATE=1
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/lbstats.txt && \
for v in ${VARIANTS:-r1abl leanabl}; do for w in ${WLS:-cfg2 cfg4}; do \
  echo "== $v $w" >> gpurun_out/lbstats.txt; \
  AIRS_LIB=exp/$v/libairscmp.so AIRS_DBG=256 timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/lbstats.txt 2>&1 || exit 1; \
done; done; grep -v amdgpu.ids gpurun_out/lbstats.txt | awk '/==/{print} /look-back stats/{n++; if (n%20==0) print}' 
