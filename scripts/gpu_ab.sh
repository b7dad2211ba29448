# GPU tests of the working tree, then A/B kernel timings of exp/base vs exp/new
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; \
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc; \
VARIANTS="${VARIANTS:-base new}" MODES=0 WLS="${WLS:-cfg2 cfg4}" bash scripts/gpu_exp.sh && python3 scripts/expres.py
