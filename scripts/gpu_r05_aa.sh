# Round 5: the C multi-GPU gather (cmp_gpu_gather) on a one-rank RCCL communicator
TAG=${1:-r05aa}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_gather_c.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -8 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
