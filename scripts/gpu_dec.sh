# decoder: GPU tests, then throughput and kernel profile
O=gpurun_out/dec
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
