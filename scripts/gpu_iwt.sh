# IWT: GPU tests (KATs, golden sequences, sizes), throughput line and kernel split
O=gpurun_out/iwt
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "kat or iwt or random or batch" > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/iwt_bench.py > $O/iwt.json 2> $O/iwt.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o iwt -- python3 scripts/iwt_bench.py > $O/kt.log 2>&1
