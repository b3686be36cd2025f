set -o pipefail
# Final-build sweep of batch sizes and metrics (bench.py, 10M x 768 f32, k=100): ms per step, kernel span, vectors/s.
cd "$GRAFT_REPO_ROOT"
for a in "--nq 1 --metric l2" "--nq 1 --metric cosine" "--nq 1 --metric inner_product" "--nq 2 --metric l2" "--nq 16 --metric l2" "--nq 64 --metric l2" "--nq 128 --metric l2" "--nq 256 --metric cosine" "--nq 256 --metric l2" "--nq 256 --metric inner_product"; do
  timeout -k 10 200 python -u bench.py $a --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bz.json 2>gpurun_out/bz.err || { echo "fail $a"; tail -5 gpurun_out/bz.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/bz.json'));print('$a', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3), round(r['value']/1e9,2), 'G vec/s')"
done
