cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "--nq 256 --metric cosine" "--nq 256 --metric l2" "--nq 2 --metric l2" "--nq 64 --metric l2" "--rows 6250000 --d 1536 --k 1000 --metric inner_product --dtype f16 --nq 256"; do
 for cap in 0 32768 65536 131072 262144; do
  if [ $cap = 0 ]; then unset FX_BATCH_CAP; else export FX_BATCH_CAP=$cap; fi
  out=$(timeout -k 10 120 python -u bench.py $cfg --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep '^{')
  rc=$?
  [ $rc -ne 0 ] && { echo "FAIL $cfg cap=$cap rc=$rc"; exit 1; }
  echo "$cfg cap=$cap $(echo "$out" | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["ms_per_step"],3), round(r["roofline"]["kernel_ms"],3))')"
 done
done
