# One call: interleaved A/B of experiment builds (VARIANTS, WLS, REPS as in
# scripts/gpu_bench_ab.sh), then scripts/gpu_r03_final.sh on the product library.
#   VARIANTS="a b" WLS="cfg3" bash scripts/gpu_r03_ab_final.sh TAG
TAG=${1:-r03_abf}
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_bench_ab.sh ${TAG}_ab || exit 1
bash scripts/gpu_r03_final.sh $TAG
