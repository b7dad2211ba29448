# pipelined kernel: GPU parity tests, then cold/warm kernel timings, pipe vs general kernel
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/exp.jsonl && \
timeout -k 10 600 python -u -m pytest tests/${TESTS:-test_gpu_parity.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/pipe_pytest.log; [ $rc -eq 0 ] || exit $rc
for p in ${PIPES:-1 0}; do for w in ${WLS:-cfg2 cfg4}; do for r in ${ROTS:-1 4}; do \
  AIRS_PIPE=$p AIRS_KB_ROT=$r timeout -k 10 120 python scripts/kbench.py $w > gpurun_out/kb.json 2>> gpurun_out/exp.err || exit 1; \
  python3 -c "import json,sys; d=json.load(open('gpurun_out/kb.json')); d['pipe']=$p; print(json.dumps(d))" >> gpurun_out/exp.jsonl; \
done; done; done; cat gpurun_out/exp.jsonl
