# A/B of build variants (exp/slw/lib_*.so: encode.hip / enc_stream.hip built
# with other -D knobs) on one bench workload (WL, default cfg2s), cold, same box.
O=gpurun_out/slw/${WL:-cfg2s}
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2; do for v in ${VARIANTS:-base w1n8 w1n32 w1s0}; do
  L=exp/slw/lib_$v.so; [ $v = base ] && L=airs-compression_amd/lib/libairscmp.so
  AIRS_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload ${WL:-cfg2s} --no-cpu-baseline --no-warm > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail -20 $O/$v.$rep.err; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('$O/$v.$rep.json'));print(d['ms_per_step'],d['roofline']['frac'],d['roofline']['achieved'],d.get('bitexact_vs_reference'))")"
done; done
