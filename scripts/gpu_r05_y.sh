# Round 5: batch + walk + autorice GPU tests (speculative fallback with separate work buffers)
TAG=${1:-r05y}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_walk.py tests/test_gpu_autorice.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head; exit $rc; }
