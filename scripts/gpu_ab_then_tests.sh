# Interleaved A/B of experiment builds (scripts/gpu_bench_ab.sh), then the
# GPU test suite on the product library.  usage: bash scripts/gpu_ab_then_tests.sh TAG
TAG=${1:-abt}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
bash scripts/gpu_bench_ab.sh $TAG || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/pytest_gpu.log | cut -c1-300
exit $rc
