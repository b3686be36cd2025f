cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
FX_IMAGE_TILED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider -k "filter_image_bit_identical or single_query_through_filter_image or batched and not contents" > gpurun_out/tiled_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/tiled_tests.log
for i in 1 2; do
 for t in 1 0; do
  for args in "--nq 256 --metric cosine" "--nq 16 --metric l2"; do
   FX_IMAGE_TILED=$t timeout -k 10 200 python -u bench.py $args --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tb.log 2>&1 || exit 1
   python -c "
import json
r = json.loads([x for x in open('gpurun_out/tb.log') if x.startswith('{')][-1])
print('tiled', $t, '$args', $i, round(r['ms_per_step'], 3), round(r['roofline']['kernel_ms'], 3))"
  done
 done
done
