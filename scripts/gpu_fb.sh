# device exact mode: batch parity tests (both modes), then the full GPU suite
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/fb && export TMPDIR=/tmp || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fb/pytest_batch.log 2>&1 || { tail -40 gpurun_out/fb/pytest_batch.log; exit 1; }
tail -3 gpurun_out/fb/pytest_batch.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fb/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/fb/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/fb/pytest_gpu.log
