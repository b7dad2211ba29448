cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
bash scripts/gpu_ablate.sh
