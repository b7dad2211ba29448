cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && : > gpurun_out/cka.jsonl || exit 1
for v in cka1 cka2; do AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 300 python scripts/ck_bench.py cfg2 >> gpurun_out/cka.jsonl 2>> gpurun_out/cka.err || exit 1; done
cat gpurun_out/cka.jsonl
