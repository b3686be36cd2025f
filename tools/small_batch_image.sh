cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for nq in 2 16 64; do
 for img in 1 0; do
  FENIX_AMD_FILTER_IMAGE=$img timeout -k 10 200 python -u bench.py --nq $nq --metric l2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sb_$nq_$img.log 2>&1 || exit 1
  python -c "
import json
r = json.loads([x for x in open('gpurun_out/sb_$nq_$img.log') if x.startswith('{')][-1])
print('nq', $nq, 'image', $img, round(r['ms_per_step'], 3), round(r['roofline']['kernel_ms'], 3))"
 done
done
