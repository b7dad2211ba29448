cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
